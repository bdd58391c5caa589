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
#include <stdlib.h>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

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

// ---- per-pixel row ops: a group of 16 lanes per pixel (4 pixels per wave) ----
// Lane l of a group handles the 4-element chunks l, l + 16, ... of the pixel's row (the
// channels of a feature map, or the window weights), so the group's loads are one
// contiguous run of the pixel's row; the row reductions are 16-lane xor shuffles.  A second
// pass re-reads the row (L1-resident) to write the outputs.
constexpr int RG = 16;

__device__ __forceinline__ float grp_sum(float v) {
  v += __shfl_xor(v, 8, RG);
  v += __shfl_xor(v, 4, RG);
  v += __shfl_xor(v, 2, RG);
  v += __shfl_xor(v, 1, RG);
  return v;
}
__device__ __forceinline__ float grp_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 8, RG));
  v = fmaxf(v, __shfl_xor(v, 4, RG));
  v = fmaxf(v, __shfl_xor(v, 2, RG));
  v = fmaxf(v, __shfl_xor(v, 1, RG));
  return v;
}

// 4 elements [e, e + 4) of a row with `len` valid entries: loads zero past len
template <typename T>
__device__ __forceinline__ f32x4 ld4(const T* row, int e, int len) {
  if (e + 4 <= len) return V4<T>::load(row + e);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < 4; ++k)
    if (e + k < len) v[k] = ld1<T>(row + e + k);
  return v;
}

// epilogue of a row chunk: entries past len are not written
template <typename T>
__device__ __forceinline__ void epi_chunk(const dvie_attn_desc& p, long long pix, int e, int len, f32x4 v) {
  if (e + 4 <= len) {
    epi4<T>(p, pix, e, v);
  } else {
    for (int k = 0; k < 4; ++k)
      if (e + k < len) epi1<T>(p, pix, e + k, v[k]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_row_kernel(const dvie_attn_desc p) {
  const long long pix = (long long)blockIdx.x * (256 / RG) + threadIdx.x / RG;
  const int l = threadIdx.x % RG;
  const long long npx = (long long)p.n * p.h * p.w;
  if (pix >= npx) return;  // whole groups leave together (the shuffles stay inside a group)
  const int K = p.wh * p.ww;
  const T* a = (const T*)p.a + pix * p.a_ld;
  const T* b0 = p.b0 ? (const T*)p.b0 + pix * p.b_ld : nullptr;
  const T* b1 = p.b1 ? (const T*)p.b1 + pix * p.b_ld : nullptr;
  switch (p.op) {
    case DVIE_ATTN_L2NORM: {
      float ss = 0.f;
      for (int e = 4 * l; e < p.c; e += 4 * RG) {
        const f32x4 v = ld4<T>(a, e, p.c);
        ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      }
      const float r = sqrtf(grp_sum(ss));
      for (int e = 4 * l; e < p.c; e += 4 * RG) {
        f32x4 v = ld4<T>(a, e, p.c);
        for (int k = 0; k < 4; ++k) v[k] = v[k] / r;
        epi_chunk<T>(p, pix, e, p.c, v);
      }
      break;
    }
    case DVIE_ATTN_L2NORM_BWD: {
      // a = dL/dxn, b0 = xn, b1 = x:  dx = (a - xn <xn, a>) / |x|
      float dot = 0.f, ss = 0.f;
      for (int e = 4 * l; e < p.c; e += 4 * RG) {
        const f32x4 g = ld4<T>(a, e, p.c), xn = ld4<T>(b0, e, p.c), x = ld4<T>(b1, e, p.c);
        for (int k = 0; k < 4; ++k) {
          dot += xn[k] * g[k];
          ss += x[k] * x[k];
        }
      }
      dot = grp_sum(dot);
      const float r = sqrtf(grp_sum(ss));
      for (int e = 4 * l; e < p.c; e += 4 * RG) {
        const f32x4 g = ld4<T>(a, e, p.c), xn = ld4<T>(b0, e, p.c);
        f32x4 v;
        for (int k = 0; k < 4; ++k) v[k] = (g[k] - xn[k] * dot) / r;
        epi_chunk<T>(p, pix, e, p.c, v);
      }
      break;
    }
    case DVIE_ATTN_SOFTMAX: {
      const int J = p.nhalf * K;
      float mx = -INFINITY;
      for (int e = 4 * l; e < J; e += 4 * RG) {
        const f32x4 v = ld4<T>(a, e, J);
        for (int k = 0; k < 4; ++k)
          if (e + k < J) mx = fmaxf(mx, v[k]);
      }
      mx = grp_max(mx);
      float s = 0.f;
      for (int e = 4 * l; e < J; e += 4 * RG) {
        const f32x4 v = ld4<T>(a, e, J);
        for (int k = 0; k < 4; ++k)
          if (e + k < J) s += expf(v[k] - mx);
      }
      const float inv = 1.f / grp_sum(s);
      for (int e = 4 * l; e < J; e += 4 * RG) {
        f32x4 v = ld4<T>(a, e, J);
        for (int k = 0; k < 4; ++k) v[k] = expf(v[k] - mx) * inv;
        epi_chunk<T>(p, pix, e, J, v);
      }
      break;
    }
    case DVIE_ATTN_SOFTMAX_BWD: {
      // a = dL/dprob, b0 = prob: dz = prob * (a - <prob, a>)
      const int J = p.nhalf * K;
      float dot = 0.f;
      for (int e = 4 * l; e < J; e += 4 * RG) {
        const f32x4 g = ld4<T>(a, e, J), pr = ld4<T>(b0, e, J);
        dot += pr[0] * g[0] + pr[1] * g[1] + pr[2] * g[2] + pr[3] * g[3];
      }
      dot = grp_sum(dot);
      for (int e = 4 * l; e < J; e += 4 * RG) {
        const f32x4 g = ld4<T>(a, e, J), pr = ld4<T>(b0, e, J);
        f32x4 v;
        for (int k = 0; k < 4; ++k) v[k] = pr[k] * (g[k] - dot);
        epi_chunk<T>(p, pix, e, J, v);
      }
      break;
    }
    case DVIE_ATTN_WNORM:
    case DVIE_ATTN_WNORM_BWD: {
      // per map m (entries [m*K, (m+1)*K)): WNORM y = a / sum(a); WNORM_BWD (a = dL/dWn,
      // b0 = Wn, b1 = W) y = (a - <a, Wn>) / sum(W)
      const bool bwd = p.op == DVIE_ATTN_WNORM_BWD;
      const int J = p.nhalf * K;
      float s0 = 0.f, s1 = 0.f, d0 = 0.f, d1 = 0.f;
      for (int e = 4 * l; e < J; e += 4 * RG) {
        const f32x4 v = ld4<T>(bwd ? b1 : a, e, J);
        f32x4 g = {0.f, 0.f, 0.f, 0.f}, wn = g;
        if (bwd) {
          g = ld4<T>(a, e, J);
          wn = ld4<T>(b0, e, J);
        }
        for (int k = 0; k < 4; ++k) {
          const bool m0 = e + k < K;
          (m0 ? s0 : s1) += v[k];
          (m0 ? d0 : d1) += g[k] * wn[k];
        }
      }
      const float inv0 = 1.f / grp_sum(s0), inv1 = 1.f / grp_sum(s1);
      if (bwd) {
        d0 = grp_sum(d0);
        d1 = grp_sum(d1);
      }
      for (int e = 4 * l; e < J; e += 4 * RG) {
        f32x4 v = ld4<T>(a, e, J);
        for (int k = 0; k < 4; ++k) {
          const bool m0 = e + k < K;
          v[k] = (v[k] - (bwd ? (m0 ? d0 : d1) : 0.f)) * (m0 ? inv0 : inv1);
        }
        epi_chunk<T>(p, pix, e, J, v);
      }
      break;
    }
    default:
      break;
  }
}

// ---- window ops on LDS tiles: one workgroup = a TP-pixel segment of one image row ----
// The (wh x ww) window of every tile pixel reads the wh source rows around it over
// TP + ww - 1 columns.  Channels go in chunks of CC; per (chunk, window row) the source row
// segment (and, for the weighted gathers, that row's window weights) is staged in LDS, so
// every source value is fetched from memory once per tile and re-read from LDS by the
// ww (GATHER / CORR) window positions that use it.  LDS pixel stride CS = CC + 4 floats (an
// odd multiple of 16 B: ds_read_b128 of consecutive pixels is conflict-free).
constexpr int TP = 64, CC = 32, CS = CC + 4, WHX = 5, WWX = 9, SPAN = TP + WWX - 1;

template <typename T>
__device__ __forceinline__ void stage_row(float* dst, const T* base, long long ld, int n, int yy, int xs, int h, int w,
                                          int c0, int c) {
  // dst[px * CS + ch] = base[n, yy, xs + px, c0 + ch], zero outside the image / past c
  const bool rowin = base && (unsigned)yy < (unsigned)h;
  for (int e = threadIdx.x; e < SPAN * (CC / 4); e += 256) {
    const int px = e / (CC / 4), q = e - px * (CC / 4);
    const int x = xs + px, ch = c0 + 4 * q;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (rowin && (unsigned)x < (unsigned)w && ch < c) v = V4<T>::load(base + (((long long)n * h + yy) * w + x) * ld + ch);
    *(f32x4*)(dst + px * CS + 4 * q) = v;
  }
}

__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3]; }

struct Tile {
  int n, y, x0;
};
__device__ __forceinline__ Tile tile_of(int w, int h) {
  const int tx = cdiv(w, TP);
  const long long r = blockIdx.x / tx;
  Tile t;
  t.x0 = (int)(blockIdx.x - r * tx) * TP;
  t.y = (int)(r % h);
  t.n = (int)(r / h);
  return t;
}

// CORR: y[p, m*K + k] = <a[p, :c], b_m[p + o_k, :c]>.  Thread = (pixel px, pair group);
// the (map, window column) pairs of each window row are spread over the 4 groups.
template <typename T>
__global__ __launch_bounds__(256) void attn_corr_tile_kernel(const dvie_attn_desc p) {
  __shared__ __attribute__((aligned(16))) float lds[TP * CS + 2 * SPAN * CS];
  float* sA = lds;
  float* sB = lds + TP * CS;
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2, J = p.nhalf * K, NP = p.nhalf * p.ww;
  const int px = threadIdx.x & (TP - 1), grp = threadIdx.x / TP;
  const T* maps[2] = {(const T*)p.b0, (const T*)p.b1};
  float acc[WHX][5];
#pragma unroll
  for (int r = 0; r < WHX; ++r)
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[r][i] = 0.f;
  for (int c0 = 0; c0 < p.c; c0 += CC) {
    __syncthreads();
    for (int e = threadIdx.x; e < TP * (CC / 4); e += 256) {  // this tile's a
      const int q = e / (CC / 4), k = e - q * (CC / 4);
      const int x = t.x0 + q, ch = c0 + 4 * k;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (x < p.w && ch < p.c) v = V4<T>::load((const T*)p.a + (((long long)t.n * p.h + t.y) * p.w + x) * p.a_ld + ch);
      *(f32x4*)(sA + q * CS + 4 * k) = v;
    }
#pragma unroll
    for (int r = 0; r < WHX; ++r) {
      if (r < p.wh) {
        if (r) __syncthreads();
        for (int m = 0; m < p.nhalf; ++m)
          stage_row<T>(sB + m * SPAN * CS, maps[m], p.b_ld, t.n, t.y + r - rh, t.x0 - rw, p.h, p.w, c0, p.c);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int pr = grp + 4 * i;
          if (pr < NP) {
            const int m = pr / p.ww, kc = pr - m * p.ww;
            const float* bp = sB + m * SPAN * CS + (px + kc) * CS;
            const float* ap = sA + px * CS;
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < CC / 4; ++q) s += dot4(*(const f32x4*)(ap + 4 * q), *(const f32x4*)(bp + 4 * q));
            acc[r][i] += s;
          }
        }
      }
    }
  }
  // outputs through LDS so that consecutive lanes write consecutive entries of a pixel row
  __syncthreads();
  float* sO = lds;  // TP x J (J <= 2 * WHX * WWX = 90 < 2 * SPAN * CS / TP)
#pragma unroll
  for (int r = 0; r < WHX; ++r)
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int pr = grp + 4 * i;
      if (r < p.wh && pr < NP) {
        const int m = pr / p.ww, kc = pr - m * p.ww;
        sO[px * J + m * K + r * p.ww + kc] = maps[m] ? acc[r][i] : 0.f;
      }
    }
  __syncthreads();
  const int npx = min(TP, p.w - t.x0);
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  for (int e = threadIdx.x; e < npx * J; e += 256) {
    const int q = e / J, j = e - q * J;
    epi1<T>(p, pix0 + q, j, sO[q * J + j]);
  }
}

// GATHER: y[p, :c] = sum_m sum_k a[p, (half0 + m) K + k] * b_m[p + o_k, :c];
// thread = (pixel, 8 channels of the chunk)
template <typename T>
__global__ __launch_bounds__(256) void attn_gather_tile_kernel(const dvie_attn_desc p) {
  constexpr int WS = 2 * WWX + 1;  // per-pixel weights of one window row (both maps), odd stride
  __shared__ __attribute__((aligned(16))) float sB[2 * SPAN * CS];
  __shared__ float sW[TP * WS];
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2;
  const int nm = p.b1 ? 2 : 1;
  const int px = threadIdx.x & (TP - 1), cg = threadIdx.x / TP;
  const T* maps[2] = {(const T*)p.b0, (const T*)p.b1};
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  const int npx = min(TP, p.w - t.x0);
  for (int c0 = 0; c0 < p.c; c0 += CC) {
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    for (int r = 0; r < p.wh; ++r) {
      __syncthreads();
      for (int m = 0; m < nm; ++m)
        stage_row<T>(sB + m * SPAN * CS, maps[m], p.b_ld, t.n, t.y + r - rh, t.x0 - rw, p.h, p.w, c0, p.c);
      for (int e = threadIdx.x; e < TP * nm * p.ww; e += 256) {
        const int q = e / (nm * p.ww), mk = e - q * (nm * p.ww);
        const int m = mk / p.ww, kc = mk - m * p.ww;
        sW[q * WS + mk] = q < npx ? ld1<T>((const T*)p.a + (pix0 + q) * p.a_ld + (p.half0 + m) * K + r * p.ww + kc) : 0.f;
      }
      __syncthreads();
      for (int m = 0; m < nm; ++m)
        for (int kc = 0; kc < p.ww; ++kc) {
          const float wk = sW[px * WS + m * p.ww + kc];
          const float* bp = sB + m * SPAN * CS + (px + kc) * CS + 8 * cg;
          acc0 += wk * *(const f32x4*)bp;
          acc1 += wk * *(const f32x4*)(bp + 4);
        }
    }
    const int ch = c0 + 8 * cg;
    if (px < npx) {
      if (ch < p.c) epi4<T>(p, pix0 + px, ch, acc0);
      if (ch + 4 < p.c) epi4<T>(p, pix0 + px, ch + 4, acc1);
    }
  }
}

// GATHER_T: y[q, :c] = sum_k a[q - o_k, half0 K + k] * b0[q - o_k, :c] (the adjoint of GATHER
// in b); staged source row r holds y + r - rh, whose window entries for q are k = (wh-1-r) ww + kc
template <typename T>
__global__ __launch_bounds__(256) void attn_gather_t_tile_kernel(const dvie_attn_desc p) {
  __shared__ __attribute__((aligned(16))) float sB[SPAN * CS];
  __shared__ float sW[SPAN * WWX];
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2;
  const int px = threadIdx.x & (TP - 1), cg = threadIdx.x / TP;
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  const int npx = min(TP, p.w - t.x0);
  const int span = TP + p.ww - 1;
  for (int c0 = 0; c0 < p.c; c0 += CC) {
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    for (int r = 0; r < p.wh; ++r) {
      const int yy = t.y + r - rh, kr = p.wh - 1 - r;
      __syncthreads();
      stage_row<T>(sB, (const T*)p.b0, p.b_ld, t.n, yy, t.x0 - rw, p.h, p.w, c0, p.c);
      for (int e = threadIdx.x; e < span * p.ww; e += 256) {
        const int s = e / p.ww, kc = e - s * p.ww;
        const int x = t.x0 - rw + s;
        float v = 0.f;
        if ((unsigned)yy < (unsigned)p.h && (unsigned)x < (unsigned)p.w)
          v = ld1<T>((const T*)p.a + (((long long)t.n * p.h + yy) * p.w + x) * p.a_ld + p.half0 * K + kr * p.ww + kc);
        sW[s * WWX + kc] = v;
      }
      __syncthreads();
      for (int kc = 0; kc < p.ww; ++kc) {
        const int s = px + p.ww - 1 - kc;
        const float wk = sW[s * WWX + kc];
        const float* bp = sB + s * CS + 8 * cg;
        acc0 += wk * *(const f32x4*)bp;
        acc1 += wk * *(const f32x4*)(bp + 4);
      }
    }
    const int ch = c0 + 8 * cg;
    if (px < npx) {
      if (ch < p.c) epi4<T>(p, pix0 + px, ch, acc0);
      if (ch + 4 < p.c) epi4<T>(p, pix0 + px, ch + 4, acc1);
    }
  }
}


// ---- GATHER on the matrix cores (bf16, c % 32 == 0, windows up to 5 x 9) ----
// For window row r and map m the tile's output is a band GEMM over the staged source row
//   y[p][ch] += sum_s W[p][s] * B[s][ch],   s = source column - (x0 - rw), 0 <= s < 64 + 2 rw,
//   W[p][s] = a[p][(half0 + m) K + r ww + (s - p)] for 0 <= s - p < ww, else 0,
// computed as D[ch][p] = B^T[ch][s] W^T[s][p] with v_mfma_f32_32x32x16_bf16: the A operand
// (32 channels x 16 sources) by transposed reads (ds_read_b64_tr_b16) of the staged rows, the
// B operand (16 sources x 32 pixels) by plain reads of the band image, whose zero entries are
// written once per workgroup (only the band positions are rewritten per window row).  A
// 32-pixel block's band spans 40 sources: 3 k-steps.  The VALU form (attn_gather_tile_kernel)
// reads every source value from LDS once per window column (9x); here the matrix cores do the
// 9-tap sums, so the LDS traffic per output drops ~3x and the window sums leave the VALU.
// Same products (bf16 x bf16 is exact in fp32); fp32 sums in another order.
constexpr int GM_TP = 64, GM_SP = 80, GM_BP = 176;  // tile pixels, staged sources, band row pitch (B)

__device__ __forceinline__ bf16x8 gm_tr_pair(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// TR: GATHER_T (the adjoint in b, one map): the band entry (q, s) is the weight of window
// entry ((wh - 1 - r), q - s + 2 rw) stored at the SOURCE pixel s, so the band is built from
// the source pixels' weight rows instead of the output pixels'.
template <bool TR>
__global__ __launch_bounds__(256) void attn_gather_mfma_kernel(const dvie_attn_desc p) {
  __shared__ __attribute__((aligned(16))) char sB[2 * GM_SP * 128];   // [m][s][64 ch], chunks swizzled
  __shared__ __attribute__((aligned(16))) char sW[2 * GM_TP * GM_BP]; // [m][p][s] band, bf16
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2;
  const int nm = p.b1 ? 2 : 1;
  const bf16_t* maps[2] = {(const bf16_t*)p.b0, (const bf16_t*)p.b1};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pb = wave & 1, cb = wave >> 1;  // 32-pixel block, 32-channel block of the chunk
  const int r32 = lane & 31, hh = lane >> 5;
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  const int npx = min(GM_TP, p.w - t.x0);

  for (int i = tid; i < 2 * GM_TP * GM_BP / 16; i += 256) ((i32x4*)sW)[i] = i32x4{0, 0, 0, 0};

  // transposed-read addressing: lane 4 q + pq of 16-lane group g4 reads source row q (+4 for
  // the second read, +8 for the upper half-wave) and 8 bytes at channel 16 (g4 & 1) + 4 pq of
  // the wave's 32 channels; the chunk swizzle c ^ 4 ((s >> 1) & 1) keeps the reads conflict-free
  const int g4 = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int tcol = 32 * cb + 16 * (g4 & 1) + 4 * tp;
  const int a_off = (tq + 8 * (g4 >> 1)) * 128 + ((((tcol >> 3) ^ (((tq >> 1) & 1) << 2))) << 4) + (tcol & 7) * 2;
  const int b_off = (32 * pb + r32) * GM_BP + hh * 16;

  // stages st = (channel chunk st / wh, window row st % wh); the next stage's source rows and
  // band weights are loaded into registers while this stage's MFMAs run (3 workgroups per CU
  // hide the rest), and written to LDS after the next barrier
  const int nstage = ((p.c + 63) / 64) * p.wh;
  i32x4 pv[2][3];
  bf16_t pw[2][3];
  auto fetch = [&](int st) {
    const int c0 = 64 * (st / p.wh), r = st % p.wh, yy = t.y + r - rh;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = tid + 256 * u, s = i >> 3, ck = i & 7;
        const int x = t.x0 - rw + s, ch = c0 + 8 * ck;
        pv[m][u] = i32x4{0, 0, 0, 0};
        if (m < nm && i < GM_SP * 8 && s < GM_TP + 2 * rw && (unsigned)yy < (unsigned)p.h && (unsigned)x < (unsigned)p.w &&
            ch < p.c)
          pv[m][u] = *(const i32x4*)(maps[m] + (((long long)t.n * p.h + yy) * p.w + x) * p.b_ld + ch);
        pw[m][u] = 0;
        if constexpr (!TR) {
          const int q = i / p.ww, kc = i - q * p.ww;
          if (m < nm && i < GM_TP * p.ww && q < npx)
            pw[m][u] = ((const bf16_t*)p.a)[(pix0 + q) * p.a_ld + (p.half0 + m) * K + r * p.ww + kc];
        } else {
          const int sx = i / p.ww, kc = i - sx * p.ww, xs = t.x0 - rw + sx;
          if (m == 0 && i < (GM_TP + 2 * rw) * p.ww && (unsigned)yy < (unsigned)p.h && (unsigned)xs < (unsigned)p.w)
            pw[m][u] = ((const bf16_t*)p.a)[(((long long)t.n * p.h + yy) * p.w + xs) * p.a_ld + p.half0 * K +
                                            (p.wh - 1 - r) * p.ww + kc];
        }
      }
    }
  };
  auto store = [&](int st) {
    const int r = st % p.wh, yy = t.y + r - rh;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (m >= nm) continue;
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = tid + 256 * u, s = i >> 3, ck = i & 7;
        if (i < GM_SP * 8) *(i32x4*)(sB + m * GM_SP * 128 + s * 128 + ((ck ^ (((s >> 1) & 1) << 2)) << 4)) = pv[m][u];
        if constexpr (!TR) {
          // band values of this window row: W[q][q + kc] = a[q][(half0 + m) K + r ww + kc]
          const int q = i / p.ww, kc = i - q * p.ww;
          if (i < GM_TP * p.ww && q < npx) *(bf16_t*)(sW + m * GM_TP * GM_BP + q * GM_BP + (q + kc) * 2) = pw[m][u];
        } else {
          // W[q][s] = a[source s][half0 K + (wh - 1 - r) ww + kc], q = s - 2 rw + kc; sources
          // outside the image are zero rows of sB, so their (stale, finite) band entries add 0
          const int sx = i / p.ww, kc = i - sx * p.ww, q = sx - 2 * rw + kc, xs = t.x0 - rw + sx;
          if (m == 0 && i < (GM_TP + 2 * rw) * p.ww && q >= 0 && q < npx && (unsigned)yy < (unsigned)p.h &&
              (unsigned)xs < (unsigned)p.w)
            *(bf16_t*)(sW + q * GM_BP + sx * 2) = pw[m][u];
        }
      }
    }
  };

  static_assert(GM_SP * 8 <= 3 * 256 && GM_TP * WWX <= 3 * 256 && (GM_TP + WWX - 1) * WWX <= 3 * 256, "prefetch slots");
  fetch(0);
  f32x16 acc = {};
  for (int st = 0; st < nstage; ++st) {
    const int c0 = 64 * (st / p.wh), r = st % p.wh;
    __syncthreads();  // the previous stage's MFMAs are done with sB / sW
    store(st);
    if (st + 1 < nstage) fetch(st + 1);
    __syncthreads();
    for (int m = 0; m < nm; ++m) {
      const char* B = sB + m * GM_SP * 128;
      const char* W = sW + m * GM_TP * GM_BP;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int s0 = 32 * pb + 16 * ks;
        const bf16x8 av = gm_tr_pair(B + a_off + s0 * 128, B + a_off + (s0 + 4) * 128);
        const i32x4 bv = *(const i32x4*)(W + b_off + s0 * 2);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
      }
    }
    if (r + 1 < p.wh) continue;
    // epilogue: permlane32 pairing -> 8 consecutive channels of one pixel per lane
    float v[2][8];
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[8 * P + e]), __float_as_uint(acc[8 * P + 4 + e]),
                                                         false, false);
        v[P][e] = __uint_as_float(sw[0]);
        v[P][4 + e] = __uint_as_float(sw[1]);
      }
    const int q = 32 * pb + r32;
    if (q < npx) {
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const int ch = c0 + 32 * cb + 16 * P + 8 * hh;
        if (ch < p.c) {
          epi4<bf16_t>(p, pix0 + q, ch, f32x4{v[P][0], v[P][1], v[P][2], v[P][3]});
          epi4<bf16_t>(p, pix0 + q, ch + 4, f32x4{v[P][4], v[P][5], v[P][6], v[P][7]});
        }
      }
    }
    acc = f32x16{};
  }
}


// ---- CORR on the matrix cores (bf16, c % 32 == 0, windows up to 5 x 9) ----
// y[p][m K + r ww + kc] = <a[p], b_m[p + (r - rh, kc - rw)]>: for map m and window row r,
// D[s][p] = sum_c B[s][c] a[p][c] over the staged source row (s = source column - (x0 - rw))
// with v_mfma_f32_32x32x16_bf16 (A operand: source rows, B operand: the tile's pixels, both
// plain row reads of XOR-swizzled 128-B rows), of which each lane keeps its band entries
// s - p in [0, ww) and adds them into an fp32 LDS row per pixel (channels go in chunks of
// 64).  Wave (pb, sb): pixel block pb, source block 32 pb + 32 sb .. +31.
constexpr int CM_TP = 64, CM_SP = 80, CM_J = 2 * WHX * WWX;

__global__ __launch_bounds__(256) void attn_corr_mfma_kernel(const dvie_attn_desc p) {
  __shared__ __attribute__((aligned(16))) char sA[CM_TP * 128];
  __shared__ __attribute__((aligned(16))) char sB[CM_SP * 128];
  __shared__ float sO[CM_TP * CM_J];
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2, J = p.nhalf * K;
  const bf16_t* maps[2] = {(const bf16_t*)p.b0, (const bf16_t*)p.b1};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pb = wave & 1, sb = wave >> 1;
  const int r32 = lane & 31, hh = lane >> 5;
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  const int npx = min(CM_TP, p.w - t.x0);
  for (int i = tid; i < CM_TP * CM_J; i += 256) sO[i] = 0.f;

  // this lane's operand rows; source rows past the staged 80 (pixel block 1, source block 1,
  // lanes >= 16) read row 79: their entries are never in a band (s - p >= 17)
  const int srow = min(32 * pb + 32 * sb + r32, CM_SP - 1), prow = 32 * pb + r32;
  // stages st = (channel chunk, live map, window row); the next stage's source row (and at a
  // chunk's first stage its pixel rows) are loaded into registers while this stage's MFMAs run
  // live maps (a missing map's entries stay zero): lm0, and lm1 when both are present
  const int nlive = (p.b0 ? 1 : 0) + (p.nhalf > 1 && p.b1 ? 1 : 0);
  const int lm0 = p.b0 ? 0 : 1, lm1 = 1;
  const int per_chunk = nlive * p.wh, nstage = ((p.c + 63) / 64) * per_chunk;
  i32x4 pv[3], pa[2];
  auto fetch = [&](int st) {
    const int c0 = 64 * (st / per_chunk), rem = st % per_chunk, m = rem / p.wh ? lm1 : lm0, r = rem % p.wh;
    const int yy = t.y + r - rh;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int i = tid + 256 * u, s = i >> 3, ck = i & 7;
      const int x = t.x0 - rw + s, ch = c0 + 8 * ck;
      pv[u] = i32x4{0, 0, 0, 0};
      if (i < CM_SP * 8 && s < CM_TP + 2 * rw && (unsigned)yy < (unsigned)p.h && (unsigned)x < (unsigned)p.w && ch < p.c)
        pv[u] = *(const i32x4*)(maps[m] + (((long long)t.n * p.h + yy) * p.w + x) * p.b_ld + ch);
    }
    if (rem == 0) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u, q = i >> 3, ck = i & 7, ch = c0 + 8 * ck;
        pa[u] = i32x4{0, 0, 0, 0};
        if (q < npx && ch < p.c) pa[u] = *(const i32x4*)((const bf16_t*)p.a + (pix0 + q) * p.a_ld + ch);
      }
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int i = tid + 256 * u, s = i >> 3, ck = i & 7;
      if (i < CM_SP * 8) *(i32x4*)(sB + s * 128 + ((ck ^ ((s >> 1) & 7)) << 4)) = pv[u];
    }
    if (st % per_chunk == 0) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u, q = i >> 3, ck = i & 7;
        *(i32x4*)(sA + q * 128 + ((ck ^ ((q >> 1) & 7)) << 4)) = pa[u];
      }
    }
  };
  static_assert(CM_SP * 8 <= 3 * 256 && CM_TP * 8 == 2 * 256, "prefetch slots");
  if (nstage > 0) fetch(0);
  for (int st = 0; st < nstage; ++st) {
    const int rem = st % per_chunk, m = rem / p.wh ? lm1 : lm0, r = rem % p.wh;
    __syncthreads();  // sO zeroed / the previous stage's reads of sA / sB are done
    store(st);
    if (st + 1 < nstage) fetch(st + 1);
    __syncthreads();
    f32x16 acc = {};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int ck = 2 * ks + hh;
      const i32x4 av = *(const i32x4*)(sB + srow * 128 + ((ck ^ ((srow >> 1) & 7)) << 4));
      const i32x4 bv = *(const i32x4*)(sA + prow * 128 + ((ck ^ ((prow >> 1) & 7)) << 4));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv), acc,
                                                    0, 0, 0);
    }
    // lane: pixel prow (column), sources 32 pb + 32 sb + 8 (e / 4) + 4 hh + e % 4 (rows)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int s = 32 * pb + 32 * sb + 8 * (e >> 2) + 4 * hh + (e & 3);
      const int kc = s - prow;
      if (kc >= 0 && kc < p.ww) sO[prow * CM_J + m * K + r * p.ww + kc] += acc[e];
    }
  }
  __syncthreads();
  for (int e = tid; e < npx * J; e += 256) {
    const int q = e / J, j = e - q * J;
    epi1<bf16_t>(p, pix0 + q, j, sO[q * CM_J + j]);
  }
}

// ---- CORR in one-barrier stages for c <= 128 (the refinement nets' 128-channel features) ----
// attn_corr_mfma_kernel stages one (64-channel chunk, window row) per stage behind two
// barriers and adds every chunk's band into its LDS rows.  Here K = channels runs over ALL
// channels inside a stage (two 64-channel planes of 128-B rows), so a stage is one (map,
// window row), its band entries are complete after its MFMAs and are written (not added) to
// the LDS output rows; the source rows are double-buffered in LDS, one barrier per stage.
// C5 (profiles/r05o/): corr 0.212 -> 0.159 ms, the prob gradient 0.143 -> 0.102.  Measured
// dead ends: the same one-barrier form of GATHER / GATHER_T (all channels and one map per
// stage, 63.5 KB: gathers 0.358 -> 0.475 ms), loads two stages ahead (two register sets) in
// both kernels, and XCD-contiguous tile ranges (gathers 0.475 -> 0.443 but CORR 0.159 ->
// 0.188 and the gradients' gathers 1.139 -> 1.253).
constexpr int A2_CP = 2;                                          // channel planes: c <= 128
constexpr int A2_SB = A2_CP * CM_SP * 128;                        // staged source row, all planes

constexpr int A2_CA = A2_CP * CM_TP * 128;  // the tile's pixel rows, all planes
static_assert(A2_CA + 2 * A2_SB + CM_TP * CM_J * 4 <= 81920, "two corr workgroups per CU");

__global__ __launch_bounds__(256, 2) void attn_corr_mfma2_kernel(const dvie_attn_desc p) {
  __shared__ __attribute__((aligned(16))) char sA[A2_CA];
  __shared__ __attribute__((aligned(16))) char sB[2 * A2_SB];
  __shared__ float sO[CM_TP * CM_J];
  const Tile t = tile_of(p.w, p.h);
  const int K = p.wh * p.ww, rh = p.wh / 2, rw = p.ww / 2, J = p.nhalf * K;
  const bf16_t* maps[2] = {(const bf16_t*)p.b0, (const bf16_t*)p.b1};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pb = wave & 1, sb = wave >> 1;
  const int r32 = lane & 31, hh = lane >> 5;
  const long long pix0 = ((long long)t.n * p.h + t.y) * p.w + t.x0;
  const int npx = min(CM_TP, p.w - t.x0);
  const int ncp = (p.c + 63) / 64;
  const int srow = min(32 * pb + 32 * sb + r32, CM_SP - 1), prow = 32 * pb + r32;
  // live maps (a missing map's entries are written as zeros): lm0, and lm1 when both are present
  const bool live1 = p.nhalf > 1 && p.b1;
  const int nlive = (p.b0 ? 1 : 0) + (live1 ? 1 : 0);
  const int lm0 = p.b0 ? 0 : 1;
  const int nstage = nlive * p.wh;
  i32x4 pv[5];
  auto fetch = [&](int st) {
    const int m = st / p.wh ? 1 : lm0, r = st % p.wh, yy = t.y + r - rh;
    const bool rowin = (unsigned)yy < (unsigned)p.h;
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = tid + 256 * u, s = i >> 4, ck = i & 15;
      const int x = t.x0 - rw + s, ch = 8 * ck;
      pv[u] = i32x4{0, 0, 0, 0};
      if (s < CM_TP + 2 * rw && rowin && (unsigned)x < (unsigned)p.w && ch < p.c)
        pv[u] = *(const i32x4*)(maps[m] + (((long long)t.n * p.h + yy) * p.w + x) * p.b_ld + ch);
    }
  };
  auto store = [&](int buf) {
    char* B = sB + buf * A2_SB;
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = tid + 256 * u, s = i >> 4, ck = i & 15, pl = ck >> 3, c8 = ck & 7;
      *(i32x4*)(B + pl * CM_SP * 128 + s * 128 + ((c8 ^ ((s >> 1) & 7)) << 4)) = pv[u];
    }
  };
  // the tile's pixel rows (all channels), once
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + 256 * u, q = i >> 4, ck = i & 15, pl = ck >> 3, c8 = ck & 7, ch = 8 * ck;
    i32x4 v = {0, 0, 0, 0};
    if (q < npx && ch < p.c) v = *(const i32x4*)((const bf16_t*)p.a + (pix0 + q) * p.a_ld + ch);
    *(i32x4*)(sA + pl * CM_TP * 128 + q * 128 + ((c8 ^ ((q >> 1) & 7)) << 4)) = v;
  }
  if (nstage > 0) {
    fetch(0);
    store(0);
  }
  __syncthreads();
  // stage st: compute from buffer st & 1, the next stage's rows loaded into registers under
  // the MFMAs and written to the other buffer (its last readers passed the previous barrier)
  for (int st = 0; st < nstage; ++st) {
    const int m = st / p.wh ? 1 : lm0, r = st % p.wh;
    if (st + 1 < nstage) fetch(st + 1);
    const char* B = sB + (st & 1) * A2_SB;
    f32x16 acc = {};
#pragma unroll
    for (int pl = 0; pl < A2_CP; ++pl) {
      if (pl >= ncp) continue;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ck = 2 * ks + hh;
        const i32x4 av = *(const i32x4*)(B + pl * CM_SP * 128 + srow * 128 + ((ck ^ ((srow >> 1) & 7)) << 4));
        const i32x4 bv = *(const i32x4*)(sA + pl * CM_TP * 128 + prow * 128 + ((ck ^ ((prow >> 1) & 7)) << 4));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv), acc,
                                                      0, 0, 0);
      }
    }
    // lane: pixel prow (column), sources 32 pb + 32 sb + 8 (e / 4) + 4 hh + e % 4 (rows); each
    // band entry (s - prow in [0, ww)) belongs to exactly one lane of one wave
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int s = 32 * pb + 32 * sb + 8 * (e >> 2) + 4 * hh + (e & 3);
      const int kc = s - prow;
      if (kc >= 0 && kc < p.ww) sO[prow * CM_J + m * K + r * p.ww + kc] = acc[e];
    }
    if (st + 1 < nstage) store((st + 1) & 1);
    __syncthreads();
  }
  // outputs: (pixel, entry) pairs advanced by 256 without divisions
  int q = tid / J, j = tid - (tid / J) * J;
  const int dq = 256 / J, dj = 256 - dq * J;
  for (int e = tid; e < npx * J; e += 256) {
    const bool live = j < K ? p.b0 != nullptr : live1;
    epi1<bf16_t>(p, pix0 + q, j, live ? sO[q * CM_J + j] : 0.f);
    q += dq;
    j += dj;
    if (j >= J) {
      j -= J;
      ++q;
    }
  }
}

}  // namespace dvie

using namespace dvie;

// DVIE_ATTN_MFMA (A/B runs, read per launch): 0 = the VALU window kernels for GATHER /
// GATHER_T / CORR, 2 = the chunked two-barrier CORR kernel at every channel count
static int gm_mode() {
  const char* e = getenv("DVIE_ATTN_MFMA");
  return e && *e == '0' ? 0 : e && *e == '2' ? 2 : 1;
}
static bool gm_on() { return gm_mode() != 0; }

extern "C" int dvie_attn(const dvie_attn_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->a && d->y, "attn: null pointer");
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0, "attn: empty shape");
  DVIE_CHECK_ARG(d->wh >= 1 && d->ww >= 1 && (d->wh & 1) && (d->ww & 1), "attn: window %dx%d must be odd",
                 d->wh, d->ww);
  DVIE_CHECK_ARG(d->dtype == DVIE_F32 || d->dtype == DVIE_BF16, "attn: dtype");
  DVIE_CHECK_ARG(!d->dact || d->z, "attn: dact needs z");
  DVIE_CHECK_ARG(d->a_ld % 4 == 0 && d->y_ld % 4 == 0 && ((!d->b0 && !d->b1) || d->b_ld % 4 == 0) &&
                     (!d->res || d->res_ld % 4 == 0) && (!d->z || d->z_ld % 4 == 0),
                 "attn: every ld must be a multiple of 4");
  const int K = d->wh * d->ww;
  const long long npx = (long long)d->n * d->h * d->w;
  const bool bf = d->dtype == DVIE_BF16;
  hipStream_t s = (hipStream_t)stream;
  // the LDS-tiled window kernels cover windows up to WHX x WWX (the refinement nets' 5 x 9)
  const bool tiled = d->wh <= WHX && d->ww <= WWX;
  const long long tiles = (long long)d->n * d->h * cdiv(d->w, TP);
  switch (d->op) {
    case DVIE_ATTN_GATHER:
    case DVIE_ATTN_GATHER_T:
    case DVIE_ATTN_POOL:
    case DVIE_ATTN_POOL_T: {
      DVIE_CHECK_ARG(d->c > 0 && d->c % 4 == 0, "attn: c=%d must be a multiple of 4", d->c);
      if (d->op == DVIE_ATTN_GATHER || d->op == DVIE_ATTN_GATHER_T) {
        DVIE_CHECK_ARG(d->b0, "attn: gather needs b0");
        DVIE_CHECK_ARG(d->half0 >= 0 && d->half0 + (d->b1 ? 2 : 1) <= d->nhalf && d->a_ld >= d->nhalf * K,
                       "attn: gather half0=%d nhalf=%d", d->half0, d->nhalf);
        DVIE_CHECK_ARG(d->op == DVIE_ATTN_GATHER || !d->b1, "attn: gather_t takes one map");
      }
      if ((d->op == DVIE_ATTN_GATHER || d->op == DVIE_ATTN_GATHER_T) && tiled && bf && d->c % 32 == 0 &&
          d->b_ld % 8 == 0 && gm_on()) {
        if (d->op == DVIE_ATTN_GATHER)
          DVIE_LAUNCH(attn_gather_mfma_kernel<false>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        else
          DVIE_LAUNCH(attn_gather_mfma_kernel<true>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        break;
      }
      if (tiled && d->op == DVIE_ATTN_GATHER) {
        if (bf)
          DVIE_LAUNCH(attn_gather_tile_kernel<bf16_t>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        else
          DVIE_LAUNCH(attn_gather_tile_kernel<float>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        break;
      }
      if (tiled && d->op == DVIE_ATTN_GATHER_T) {
        if (bf)
          DVIE_LAUNCH(attn_gather_t_tile_kernel<bf16_t>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        else
          DVIE_LAUNCH(attn_gather_t_tile_kernel<float>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        break;
      }
      const long long tot = npx * (d->c / 4);
      const dim3 grid((unsigned)((tot + 255) / 256));
      if (bf)
        DVIE_LAUNCH(attn_vec_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
      else
        DVIE_LAUNCH(attn_vec_kernel<float>, grid, dim3(256), 0, s, *d);
      break;
    }
    case DVIE_ATTN_CORR: {
      DVIE_CHECK_ARG((d->nhalf == 1 || d->nhalf == 2) && (d->b0 || d->b1), "attn: corr maps");
      DVIE_CHECK_ARG(d->c > 0 && d->c % 4 == 0, "attn: corr c=%d", d->c);
      DVIE_CHECK_ARG(d->y_ld >= d->nhalf * K, "attn: corr y_ld");
      if (tiled && bf && d->c % 32 == 0 && d->a_ld % 8 == 0 && d->b_ld % 8 == 0 && gm_on()) {
        if (d->c <= 64 * A2_CP && gm_mode() == 1)
          DVIE_LAUNCH(attn_corr_mfma2_kernel, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        else
          DVIE_LAUNCH(attn_corr_mfma_kernel, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        break;
      }
      if (tiled) {
        if (bf)
          DVIE_LAUNCH(attn_corr_tile_kernel<bf16_t>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        else
          DVIE_LAUNCH(attn_corr_tile_kernel<float>, dim3((unsigned)tiles), dim3(256), 0, s, *d);
        break;
      }
      const long long tot = npx * d->nhalf * K;
      const dim3 grid((unsigned)((tot + 255) / 256));
      if (bf)
        DVIE_LAUNCH(attn_corr_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
      else
        DVIE_LAUNCH(attn_corr_kernel<float>, grid, dim3(256), 0, s, *d);
      break;
    }
    default: {
      DVIE_CHECK_ARG(d->op == DVIE_ATTN_L2NORM || d->op == DVIE_ATTN_L2NORM_BWD || d->op == DVIE_ATTN_SOFTMAX ||
                         d->op == DVIE_ATTN_SOFTMAX_BWD || d->op == DVIE_ATTN_WNORM || d->op == DVIE_ATTN_WNORM_BWD,
                     "attn: unknown op %d", d->op);
      if (d->op == DVIE_ATTN_L2NORM_BWD || d->op == DVIE_ATTN_WNORM_BWD)
        DVIE_CHECK_ARG(d->b0 && d->b1, "attn: backward needs b0 and b1");
      if (d->op == DVIE_ATTN_SOFTMAX_BWD) DVIE_CHECK_ARG(d->b0, "attn: softmax backward needs b0");
      if (d->op == DVIE_ATTN_WNORM || d->op == DVIE_ATTN_WNORM_BWD)
        DVIE_CHECK_ARG(d->nhalf == 1 || d->nhalf == 2, "attn: wnorm takes one or two maps");
      const dim3 grid((unsigned)((npx + (256 / RG) - 1) / (256 / RG)));
      if (bf)
        DVIE_LAUNCH(attn_row_kernel<bf16_t>, grid, dim3(256), 0, s, *d);
      else
        DVIE_LAUNCH(attn_row_kernel<float>, grid, dim3(256), 0, s, *d);
    }
  }
  DVIE_RETURN_LAUNCH();
}
