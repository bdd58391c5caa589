// sn.hip — SpectralNorm of the SN discriminators (reference nets/SpectralNorm.py:10-68,
// used by FrameSN* in nets/FrameDisc.py:116-189 and VideoSN* in nets/VidDisc.py:140-226).
//
// Per layer: the (h, width) weight matrix W_bar, persistent vectors u (h) and v (width).
// Forward = SpectralNorm._update_u_v (power iteration, sigma, w_eff = W_bar / sigma) with u,
// v updated in place and the values used saved for the backward; backward = the autograd of
// `w / sigma`, sigma = u . (W_bar v).  The matrices are tiny (<= 256 x 2304), so one
// 256-thread workgroup owns a layer and every reduction is done in fp64 inside it: no
// atomics, deterministic.  All layers of a discriminator go in one launch.
#include "common.h"

namespace dvie {

constexpr int SN_THREADS = 256;
constexpr int SN_BATCH = 16;  // layers per launch (descriptors passed by value)
struct SnBatch {
  dvie_sn_layer l[SN_BATCH];
};

// sum over the workgroup
__device__ double sn_block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();  // red is reusable
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < SN_THREADS / 64; ++k) s += red[k];
  return s;
}

// dst[i] = sum_j W[i][j] x[j]: one wave per row (rows wave, wave + 4, ...), lanes over j
__device__ void sn_rows(const float* __restrict__ W, const float* x, float* dst, int h, int width) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = wave; i < h; i += SN_THREADS / 64) {
    const float* row = W + (long long)i * width;
    double s = 0.0;
    for (int j = lane; j < width; j += 64) s += (double)row[j] * (double)x[j];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) dst[i] = (float)s;
  }
}

// dst[j] = sum_i W[i][j] x[i]: threads over columns, so each row read is coalesced
__device__ void sn_cols(const float* __restrict__ W, const float* x, float* dst, int h, int width) {
  for (int j = threadIdx.x; j < width; j += SN_THREADS) {
    double s = 0.0;
    for (int i = 0; i < h; ++i) s += (double)W[(long long)i * width + j] * (double)x[i];
    dst[j] = (float)s;
  }
}

// x = x / (|x| + 1e-12) in place (l2normalize, SpectralNorm.py:10-11)
__device__ void sn_normalize(float* x, int n, double* red) {
  double s = 0.0;
  for (int k = threadIdx.x; k < n; k += SN_THREADS) s += (double)x[k] * (double)x[k];
  const float nrm = (float)sqrt(sn_block_sum(s, red));
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += SN_THREADS) x[k] = x[k] / (nrm + 1e-12f);
  __syncthreads();
}

__global__ void __launch_bounds__(SN_THREADS) sn_fwd_kernel(SnBatch b, float* __restrict__ state) {
  const dvie_sn_layer L = b.l[blockIdx.x];
  extern __shared__ float sn_smem[];
  __shared__ double red[SN_THREADS / 64];
  float* vs = sn_smem;       // v (width)
  float* us = vs + L.width;  // u (h)
  float* wv = us + L.h;      // W v (h)
  for (int k = threadIdx.x; k < L.h; k += SN_THREADS) us[k] = L.u[k];
  for (int k = threadIdx.x; k < L.width; k += SN_THREADS) vs[k] = L.v[k];
  __syncthreads();
  for (int it = 0; it < L.power_iterations; ++it) {
    sn_cols(L.w_bar, us, vs, L.h, L.width);  // v = W^T u
    __syncthreads();
    sn_normalize(vs, L.width, red);
    sn_rows(L.w_bar, vs, us, L.h, L.width);  // u = W v
    __syncthreads();
    sn_normalize(us, L.h, red);
  }
  sn_rows(L.w_bar, vs, wv, L.h, L.width);  // sigma = u . (W v)
  __syncthreads();
  double s = 0.0;
  for (int k = threadIdx.x; k < L.h; k += SN_THREADS) s += (double)us[k] * (double)wv[k];
  const float sigma = (float)sn_block_sum(s, red);
  float* st = state + L.state_off;
  if (threadIdx.x == 0) st[0] = sigma;
  for (int k = threadIdx.x; k < L.h; k += SN_THREADS) {
    L.u[k] = us[k];
    st[1 + k] = us[k];
  }
  for (int k = threadIdx.x; k < L.width; k += SN_THREADS) {
    L.v[k] = vs[k];
    st[1 + L.h + k] = vs[k];
  }
  const long long n = (long long)L.h * L.width;
  for (long long e = threadIdx.x; e < n; e += SN_THREADS) L.w_eff[e] = L.w_bar[e] / sigma;
}

__global__ void __launch_bounds__(SN_THREADS) sn_bwd_kernel(SnBatch b, const float* __restrict__ state) {
  const dvie_sn_layer L = b.l[blockIdx.x];
  extern __shared__ float sn_smem[];
  __shared__ double red[SN_THREADS / 64];
  const float* st = state + L.state_off;
  const float sigma = st[0];
  const float* us = st + 1;
  const float* vs = us + L.h;
  const long long n = (long long)L.h * L.width;
  double s = 0.0;
  for (long long e = threadIdx.x; e < n; e += SN_THREADS) s += (double)L.g_eff[e] * (double)L.w_bar[e];
  // div backward: d(w / sigma)/dsigma = -sum(g * w) / sigma^2
  const float gs = (float)(-sn_block_sum(s, red) / ((double)sigma * (double)sigma));
  for (long long e = threadIdx.x; e < n; e += SN_THREADS) {
    const int i = (int)(e / L.width), j = (int)(e - (long long)i * L.width);
    const float val = L.g_eff[e] / sigma + gs * us[i] * vs[j];
    L.g_bar[e] = L.beta ? L.g_bar[e] + val : val;
  }
  if (L.g_u) {  // dsigma/du = W v
    float* wv = sn_smem;
    sn_rows(L.w_bar, vs, wv, L.h, L.width);
    __syncthreads();
    for (int k = threadIdx.x; k < L.h; k += SN_THREADS) L.g_u[k] = (L.beta ? L.g_u[k] : 0.f) + gs * wv[k];
  }
  if (L.g_v) {  // dsigma/dv = W^T u
    float* wtu = sn_smem + L.h;
    sn_cols(L.w_bar, us, wtu, L.h, L.width);
    for (int j = threadIdx.x; j < L.width; j += SN_THREADS) L.g_v[j] = (L.beta ? L.g_v[j] : 0.f) + gs * wtu[j];
  }
}

static int sn_launch(const dvie_sn_layer* layers, int n, const float* state, hipStream_t st, int bwd) {
  DVIE_CHECK_ARG(layers && n >= 0 && state, "sn: args");
  for (int i = 0; i < n; ++i) {
    const dvie_sn_layer& l = layers[i];
    DVIE_CHECK_ARG(l.w_bar && l.h > 0 && l.width > 0 && l.state_off >= 0, "sn layer %d: shape", i);
    DVIE_CHECK_ARG((l.h + 2LL * l.width) * 4 <= 65536, "sn layer %d: h %d width %d exceed the LDS vectors", i, l.h,
                   l.width);
    if (!bwd)
      DVIE_CHECK_ARG(l.u && l.v && l.w_eff && l.power_iterations >= 0, "sn fwd layer %d: pointers", i);
    else
      DVIE_CHECK_ARG(l.g_eff && l.g_bar, "sn bwd layer %d: pointers", i);
  }
  for (int i0 = 0; i0 < n; i0 += SN_BATCH) {
    SnBatch b;
    const int cnt = n - i0 < SN_BATCH ? n - i0 : SN_BATCH;
    size_t lds = 0;
    for (int k = 0; k < cnt; ++k) {
      b.l[k] = layers[i0 + k];
      const size_t need = (size_t)(b.l[k].width + 2 * b.l[k].h) * sizeof(float);
      if (need > lds) lds = need;
    }
    if (bwd)
      DVIE_LAUNCH(sn_bwd_kernel, dim3(cnt), dim3(SN_THREADS), lds, st, b, state);
    else
      DVIE_LAUNCH(sn_fwd_kernel, dim3(cnt), dim3(SN_THREADS), lds, st, b, (float*)state);
  }
  return DVIE_OK;
}

}  // namespace dvie

using namespace dvie;

extern "C" {

int dvie_sn_fwd(const dvie_sn_layer* layers, int n, float* state, void* stream) {
  const int rc = sn_launch(layers, n, state, (hipStream_t)stream, 0);
  if (rc) return rc;
  DVIE_RETURN_LAUNCH();
}

int dvie_sn_bwd(const dvie_sn_layer* layers, int n, const float* state, void* stream) {
  const int rc = sn_launch(layers, n, state, (hipStream_t)stream, 1);
  if (rc) return rc;
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"
