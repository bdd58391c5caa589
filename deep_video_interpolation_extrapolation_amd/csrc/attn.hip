// Local-window attention kernels of the second-stage refinement nets (gfx950):
// channel L2 normalisation, the local correlation volume, softmax / per-map normalisation
// of the window weights, the weighted neighbour gather and its adjoint, and the 3x5
// average pooling of the weights (stage3_prop), each with its backward.
//
// Reference: MSResAttnRefine (nets/refine_nets.py:138-399): corrmap l.253-287
// (x / x.norm, F.pad + unfold into (h=5) x (w=9) windows, sum over channels, softmax over
// both maps' 2*45 entries, avg_pool2d((3,5), pad (1,2), count_include_pad=False)),
// weight_neighbors_by_probmap l.313-323 and weight_neighbors_by_low_probmap l.289-311.
//
// Layout: NHWC, element (n, y, x, ch) at base[((n*h + y)*w + x)*ld + ch].  Window k of
// a (wh x ww) window is offset (k / ww - wh/2, k % ww - ww/2); window weights of map m
// live in channel m*wh*ww + k.  Out-of-image neighbours are zero (the reference's zero
// F.pad).  Every op ends with the engine's common epilogue:
//   v += res; v += y_old (beta); v = act(v); v *= act'(z) (dact); y = v.
#include "common.h"

namespace dvie {

template <typename T>
__device__ __forceinline__ float ld1(const T* p) {
  if constexpr (sizeof(T) == 2)
    return bf2f(*p);
  else
    return *p;
}
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (sizeof(T) == 2)
    *p = f2bf(v);
  else
    *p = v;
}

template <typename T>
__device__ __forceinline__ void epi1(const dvie_attn_desc& p, long long pix, int ch, float v) {
  T* y = (T*)p.y + pix * p.y_ld + ch;
  if (p.res) v += ld1<T>((const T*)p.res + pix * p.res_ld + ch);
  if (p.beta) v += ld1<T>(y);
  if (p.act) v = act_fwd(v, p.act, p.alpha);
  if (p.dact) v *= act_dz(ld1<T>((const T*)p.z + pix * p.z_ld + ch), p.dact, p.alpha);
  st1<T>(y, v);
}

template <typename T>
__device__ __forceinline__ void epi4(const dvie_attn_desc& p, long long pix, int ch, f32x4 v) {
  T* y = (T*)p.y + pix * p.y_ld + ch;
  if (p.res) v += V4<T>::load((const T*)p.res + pix * p.res_ld + ch);
  if (p.beta) v += V4<T>::load(y);
  if (p.act)
    for (int k = 0; k < 4; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
  if (p.dact) {
    const f32x4 z = V4<T>::load((const T*)p.z + pix * p.z_ld + ch);
    for (int k = 0; k < 4; ++k) v[k] *= act_dz(z[k], p.dact, p.alpha);
  }
  V4<T>::store(y, v);
}

struct Pix {
  int n, y, x;
};
__device__ __forceinline__ Pix unpix(long long pix, int h, int w) {
  Pix r;
  r.x = (int)(pix % w);
  const long long t = pix / w;
  r.y = (int)(t % h);
  r.n = (int)(t / h);
  return r;
}

// ---- channel-vector ops: one thread = 4 channels of one pixel ----
template <typename T>
__global__ __launch_bounds__(256) void attn_vec_kernel(const dvie_attn_desc p) {
  const int cq = p.c / 4;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long npx = (long long)p.n * p.h * p.w;
  if (e >= npx * cq) return;
  const long long pix = e / cq;
  const int ch = (int)(e - pix * cq) * 4;
  const Pix q = unpix(pix, p.h, p.w);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2;
  const T* a = (const T*)p.a;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  switch (p.op) {
    case DVIE_ATTN_GATHER: {
      // y[p] = sum_m sum_k a[p, (half0+m)*K + k] * b_m[p + o_k]
      const int nm = p.b1 ? 2 : 1;
      for (int m = 0; m < nm; ++m) {
        const T* b = (const T*)(m == 0 ? p.b0 : p.b1);
        const T* wrow = a + pix * p.a_ld + (long long)(p.half0 + m) * K;
        for (int k = 0; k < K; ++k) {
          const int yy = q.y + k / p.ww - rh, xx = q.x + k % p.ww - rw;
          if ((unsigned)yy >= (unsigned)p.h || (unsigned)xx >= (unsigned)p.w) continue;
          const float wk = ld1<T>(wrow + k);
          const f32x4 t = V4<T>::load(b + (((long long)q.n * p.h + yy) * p.w + xx) * p.b_ld + ch);
          v += wk * t;
        }
      }
      break;
    }
    case DVIE_ATTN_GATHER_T: {
      // y[q] = sum_k a[q - o_k, half0*K + k] * b0[q - o_k]
      const T* b = (const T*)p.b0;
      for (int k = 0; k < K; ++k) {
        const int yy = q.y - (k / p.ww - rh), xx = q.x - (k % p.ww - rw);
        if ((unsigned)yy >= (unsigned)p.h || (unsigned)xx >= (unsigned)p.w) continue;
        const long long src = ((long long)q.n * p.h + yy) * p.w + xx;
        const float wk = ld1<T>(a + src * p.a_ld + (long long)p.half0 * K + k);
        v += wk * V4<T>::load(b + src * p.b_ld + ch);
      }
      break;
    }
    case DVIE_ATTN_POOL: {
      // mean over the in-image part of the centred (wh x ww) window
      int cnt = 0;
      for (int i = -rh; i <= rh; ++i)
        for (int j = -rw; j <= rw; ++j) {
          const int yy = q.y + i, xx = q.x + j;
          if ((unsigned)yy >= (unsigned)p.h || (unsigned)xx >= (unsigned)p.w) continue;
          v += V4<T>::load(a + (((long long)q.n * p.h + yy) * p.w + xx) * p.a_ld + ch);
          ++cnt;
        }
      v *= 1.f / (float)cnt;
      break;
    }
    case DVIE_ATTN_POOL_T: {
      // adjoint: y[q] = sum over windows (centre s) containing q of a[s] / count(s)
      for (int i = -rh; i <= rh; ++i)
        for (int j = -rw; j <= rw; ++j) {
          const int yy = q.y + i, xx = q.x + j;
          if ((unsigned)yy >= (unsigned)p.h || (unsigned)xx >= (unsigned)p.w) continue;
          const int ch_ = min(yy + rh, p.h - 1) - max(yy - rh, 0) + 1;
          const int cw_ = min(xx + rw, p.w - 1) - max(xx - rw, 0) + 1;
          v += V4<T>::load(a + (((long long)q.n * p.h + yy) * p.w + xx) * p.a_ld + ch) * (1.f / (float)(ch_ * cw_));
        }
      break;
    }
    default:
      return;
  }
  epi4<T>(p, pix, ch, v);
}

// ---- correlation volume: one thread = one (pixel, map, window entry) ----
template <typename T>
__global__ __launch_bounds__(256) void attn_corr_kernel(const dvie_attn_desc p) {
  const int K = p.wh * p.ww, J = p.nhalf * K;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long npx = (long long)p.n * p.h * p.w;
  if (e >= npx * J) return;
  const long long pix = e / J;
  const int j = (int)(e - pix * J);
  const int m = j / K, k = j - m * K;
  const Pix q = unpix(pix, p.h, p.w);
  const int yy = q.y + k / p.ww - p.wh / 2, xx = q.x + k % p.ww - p.ww / 2;
  float s = 0.f;
  const T* bm = (const T*)(m == 0 ? p.b0 : p.b1);  // NULL map: its entries are zero
  if (bm && (unsigned)yy < (unsigned)p.h && (unsigned)xx < (unsigned)p.w) {
    const T* a = (const T*)p.a + pix * p.a_ld;
    const T* b = bm + (((long long)q.n * p.h + yy) * p.w + xx) * p.b_ld;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < p.c; c += 4) acc += V4<T>::load(a + c) * V4<T>::load(b + c);
    s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  epi1<T>(p, pix, j, s);
}

// ---- per-pixel row ops: one thread = one pixel ----
template <typename T>
__global__ __launch_bounds__(256) void attn_row_kernel(const dvie_attn_desc p) {
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long npx = (long long)p.n * p.h * p.w;
  if (pix >= npx) return;
  const int K = p.wh * p.ww;
  const T* a = (const T*)p.a + pix * p.a_ld;
  switch (p.op) {
    case DVIE_ATTN_L2NORM: {
      float ss = 0.f;
      for (int c = 0; c < p.c; ++c) {
        const float t = ld1<T>(a + c);
        ss += t * t;
      }
      const float r = sqrtf(ss);
      for (int c = 0; c < p.c; ++c) epi1<T>(p, pix, c, ld1<T>(a + c) / r);
      break;
    }
    case DVIE_ATTN_L2NORM_BWD: {
      // a = dL/dxn, b0 = xn, b1 = x:  dx = (a - xn <xn, a>) / |x|
      const T* xn = (const T*)p.b0 + pix * p.b_ld;
      const T* x = (const T*)p.b1 + pix * p.b_ld;
      float dot = 0.f, ss = 0.f;
      for (int c = 0; c < p.c; ++c) {
        const float t = ld1<T>(x + c);
        dot += ld1<T>(xn + c) * ld1<T>(a + c);
        ss += t * t;
      }
      const float r = sqrtf(ss);
      for (int c = 0; c < p.c; ++c) epi1<T>(p, pix, c, (ld1<T>(a + c) - ld1<T>(xn + c) * dot) / r);
      break;
    }
    case DVIE_ATTN_SOFTMAX: {
      const int J = p.nhalf * K;
      float mx = -INFINITY;
      for (int j = 0; j < J; ++j) mx = fmaxf(mx, ld1<T>(a + j));
      float s = 0.f;
      for (int j = 0; j < J; ++j) s += expf(ld1<T>(a + j) - mx);
      const float inv = 1.f / s;
      for (int j = 0; j < J; ++j) epi1<T>(p, pix, j, expf(ld1<T>(a + j) - mx) * inv);
      break;
    }
    case DVIE_ATTN_SOFTMAX_BWD: {
      // a = dL/dprob, b0 = prob: dz = prob * (a - <prob, a>)
      const int J = p.nhalf * K;
      const T* pr = (const T*)p.b0 + pix * p.b_ld;
      float dot = 0.f;
      for (int j = 0; j < J; ++j) dot += ld1<T>(pr + j) * ld1<T>(a + j);
      for (int j = 0; j < J; ++j) epi1<T>(p, pix, j, ld1<T>(pr + j) * (ld1<T>(a + j) - dot));
      break;
    }
    case DVIE_ATTN_WNORM: {
      for (int m = 0; m < p.nhalf; ++m) {
        float s = 0.f;
        for (int k = 0; k < K; ++k) s += ld1<T>(a + m * K + k);
        const float inv = 1.f / s;
        for (int k = 0; k < K; ++k) epi1<T>(p, pix, m * K + k, ld1<T>(a + m * K + k) * inv);
      }
      break;
    }
    case DVIE_ATTN_WNORM_BWD: {
      // a = dL/dWn, b0 = Wn, b1 = W: per map dW = (a - <a, Wn>) / sum(W)
      const T* wn = (const T*)p.b0 + pix * p.b_ld;
      const T* w = (const T*)p.b1 + pix * p.b_ld;
      for (int m = 0; m < p.nhalf; ++m) {
        float dot = 0.f, s = 0.f;
        for (int k = 0; k < K; ++k) {
          dot += ld1<T>(a + m * K + k) * ld1<T>(wn + m * K + k);
          s += ld1<T>(w + m * K + k);
        }
        const float inv = 1.f / s;
        for (int k = 0; k < K; ++k) epi1<T>(p, pix, m * K + k, (ld1<T>(a + m * K + k) - dot) * inv);
      }
      break;
    }
    default:
      break;
  }
}

}  // namespace dvie

using namespace dvie;

extern "C" int dvie_attn(const dvie_attn_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->a && d->y, "attn: null pointer");
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0, "attn: empty shape");
  DVIE_CHECK_ARG(d->wh >= 1 && d->ww >= 1 && (d->wh & 1) && (d->ww & 1), "attn: window %dx%d must be odd",
                 d->wh, d->ww);
  DVIE_CHECK_ARG(d->dtype == DVIE_F32 || d->dtype == DVIE_BF16, "attn: dtype");
  DVIE_CHECK_ARG(!d->dact || d->z, "attn: dact needs z");
  const int K = d->wh * d->ww;
  const long long npx = (long long)d->n * d->h * d->w;
  const bool vec = d->op == DVIE_ATTN_GATHER || d->op == DVIE_ATTN_GATHER_T || d->op == DVIE_ATTN_POOL ||
                   d->op == DVIE_ATTN_POOL_T;
  hipStream_t s = (hipStream_t)stream;
  if (vec) {
    DVIE_CHECK_ARG(d->c > 0 && d->c % 4 == 0, "attn: c=%d must be a multiple of 4", d->c);
    DVIE_CHECK_ARG(d->y_ld % 4 == 0 && d->b_ld % 4 == 0 && d->a_ld % 4 == 0 && (!d->res || d->res_ld % 4 == 0) &&
                       (!d->z || d->z_ld % 4 == 0),
                   "attn: ld alignment");
    if (d->op == DVIE_ATTN_GATHER || d->op == DVIE_ATTN_GATHER_T) {
      DVIE_CHECK_ARG(d->b0, "attn: gather needs b0");
      DVIE_CHECK_ARG(d->half0 >= 0 && d->half0 + (d->b1 ? 2 : 1) <= d->nhalf && d->a_ld >= d->nhalf * K,
                     "attn: gather half0=%d nhalf=%d", d->half0, d->nhalf);
    }
    const long long tot = npx * (d->c / 4);
    const dim3 grid((unsigned)((tot + 255) / 256));
    if (d->dtype == DVIE_BF16)
      hipLaunchKernelGGL(attn_vec_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
    else
      hipLaunchKernelGGL(attn_vec_kernel<float>, grid, dim3(256), 0, s, *d);
  } else if (d->op == DVIE_ATTN_CORR) {
    DVIE_CHECK_ARG((d->nhalf == 1 || d->nhalf == 2) && (d->b0 || d->b1), "attn: corr maps");
    DVIE_CHECK_ARG(d->c > 0 && d->c % 4 == 0 && d->a_ld % 4 == 0 && d->b_ld % 4 == 0, "attn: corr c=%d", d->c);
    DVIE_CHECK_ARG(d->y_ld >= d->nhalf * K, "attn: corr y_ld");
    const long long tot = npx * d->nhalf * K;
    const dim3 grid((unsigned)((tot + 255) / 256));
    if (d->dtype == DVIE_BF16)
      hipLaunchKernelGGL(attn_corr_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
    else
      hipLaunchKernelGGL(attn_corr_kernel<float>, grid, dim3(256), 0, s, *d);
  } else {
    DVIE_CHECK_ARG(d->op == DVIE_ATTN_L2NORM || d->op == DVIE_ATTN_L2NORM_BWD || d->op == DVIE_ATTN_SOFTMAX ||
                       d->op == DVIE_ATTN_SOFTMAX_BWD || d->op == DVIE_ATTN_WNORM || d->op == DVIE_ATTN_WNORM_BWD,
                   "attn: unknown op %d", d->op);
    if (d->op == DVIE_ATTN_L2NORM_BWD || d->op == DVIE_ATTN_WNORM_BWD)
      DVIE_CHECK_ARG(d->b0 && d->b1, "attn: backward needs b0 and b1");
    if (d->op == DVIE_ATTN_SOFTMAX_BWD) DVIE_CHECK_ARG(d->b0, "attn: softmax backward needs b0");
    const dim3 grid((unsigned)((npx + 255) / 256));
    if (d->dtype == DVIE_BF16)
      hipLaunchKernelGGL(attn_row_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
    else
      hipLaunchKernelGGL(attn_row_kernel<float>, grid, dim3(256), 0, s, *d);
  }
  DVIE_RETURN_LAUNCH();
}
