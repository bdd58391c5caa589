// Store / operand-load pattern probe for the wide 1x1 epilogue (tools only, not the product):
// out[pix][256 ch] = beta[pix][...] + z[pix][...] (bf16), 32 pixels per wave, 8 x 16-B chunks
// per lane.  mode 0: the MFMA-layout epilogue pattern (instruction k: lane (r32, h) -> pixel
// r32, 16-B group 2k + h: 32 pixels x 32 B per instruction); mode 1: coalesced (instruction k:
// lane l -> pixel 4k + l / 16, group l % 16: 4 pixels x 256 B per instruction); mode 2: loads
// as mode 0, stores as mode 1.
#include <hip/hip_runtime.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void store_probe_kernel(const i32x4* __restrict__ a, const i32x4* __restrict__ b,
                                                          i32x4* __restrict__ y, long long npix, int mode) {
  const int lane = threadIdx.x & 63;
  const long long wv = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long p0 = wv * 32;
  if (p0 >= npix) return;
  i32x4 va[8], vb[8];
  long long lo[8], so[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // 256 channels = 16 groups of 16 B per pixel
    const long long m0 = (p0 + (lane & 31)) * 16 + 2 * k + (lane >> 5);
    const long long m1 = (p0 + 4 * k + (lane >> 4)) * 16 + (lane & 15);
    lo[k] = mode == 1 ? m1 : m0;  // mode 2: operand loads in the MFMA order, stores coalesced
    so[k] = mode == 0 ? m0 : m1;
    va[k] = a[lo[k]];
    vb[k] = b[lo[k]];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) y[so[k]] = va[k] + vb[k];
}

extern "C" int store_probe(const void* a, const void* b, void* y, long long npix, int mode, void* stream) {
  const long long waves = (npix + 31) / 32;
  hipLaunchKernelGGL(store_probe_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const i32x4*)a, (const i32x4*)b, (i32x4*)y, npix, mode);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
