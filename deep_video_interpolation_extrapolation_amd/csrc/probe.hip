// Dense MFMA rate probe (bench.py calibration): back-to-back v_mfma_f32_32x32x16_bf16 on
// pseudo-random operands held in registers, every SIMD of every CU busy.  Under load the
// chip holds a clock well below its 2.4 GHz maximum for bf16 MFMA on random data
// (MI355X_MICROARCH.md 'DVFS give-back'), so this measured rate -- not the 2.5 PF spec --
// is the MFMA ceiling the conv kernels can approach on the same box.
#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace dvie {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// bf16 pair from 32 random bits: sign, exponent in [-2, 1], random mantissa (values in (-4, 4))
__device__ __forceinline__ int rnd_pair(uint32_t h) {
  const uint32_t a = (h & 0x807Fu) | ((125u + ((h >> 7) & 3u)) << 7);
  const uint32_t b = ((h >> 16) & 0x807Fu) | ((125u + ((h >> 23) & 3u)) << 7);
  return (int)(a | (b << 16));
}

__global__ __launch_bounds__(256) void mfma_probe_kernel(float* out, int iters) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  i32x4 a[2], b[2];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[k][e] = rnd_pair(mix32(g * 16u + k * 4u + e));
      b[k][e] = rnd_pair(mix32(g * 16u + 8u + k * 4u + e + 0x9e3779b9u));
    }
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[j & 1]),
                                                       __builtin_bit_cast(bf16x8, b[j >> 1]), acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[(j + 1) & 1]),
                                                       __builtin_bit_cast(bf16x8, b[j & 1]), acc[j], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  out[g] = s;
}

__global__ void launch_probe_kernel() {}

}  // namespace dvie

using namespace dvie;

extern "C" int dvie_mfma_probe(float* out, int blocks, int iters, void* stream) {
  DVIE_CHECK_ARG(out && blocks > 0 && iters > 0, "mfma_probe: args");
  DVIE_LAUNCH(mfma_probe_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
  DVIE_RETURN_LAUNCH();
}

extern "C" int dvie_launch_probe(int blocks, int threads, void* stream) {
  DVIE_CHECK_ARG(blocks > 0 && threads > 0 && threads <= 1024, "launch_probe: args");
  DVIE_LAUNCH(launch_probe_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)stream);
  DVIE_RETURN_LAUNCH();
}
