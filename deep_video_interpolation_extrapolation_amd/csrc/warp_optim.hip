// Bilinear flow warp (grid_sample, zeros padding) forward/backward, the fused Adamax
// step over a flat parameter buffer, and the op-list executor / ABI helpers.
//
// Reference: FlowWrapper utils/net_utils.py:89-114 (warp / warp_back l.116-129);
// torch.optim.Adamax at runners/InterTrainer.py:79.
#include "common.h"

namespace dvie {

// torch.linspace(-1, 1, n)[i] as computed by the CPU kernel (two-sided)
__device__ __forceinline__ float linspace_pm1(int i, int n) {
  if (n <= 1) return -1.f;
  const float step = 2.f / (float)(n - 1);
  return (i < n / 2) ? -1.f + step * (float)i : 1.f - step * (float)(n - 1 - i);
}

__device__ __forceinline__ float unnorm(float g, int size, int ac) {
  return ac ? ((g + 1.f) / 2.f) * (float)(size - 1) : ((g + 1.f) * (float)size - 1.f) / 2.f;
}

struct WarpTap {
  int x0, y0;
  float ix, iy, wnw, wne, wsw, wse;
  bool vx0, vx1, vy0, vy1;
};

// grid_sample's source position and bilinear corner weights for output pixel (x, y)
__device__ __forceinline__ WarpTap warp_tap(int x, int y, float fx, float fy, int w, int h, int ac) {
  WarpTap t;
  const float gx = linspace_pm1(x, w) - fx;
  const float gy = linspace_pm1(y, h) - fy;
  t.ix = unnorm(gx, w, ac);
  t.iy = unnorm(gy, h, ac);
  t.x0 = (int)floorf(t.ix);
  t.y0 = (int)floorf(t.iy);
  const int x1 = t.x0 + 1, y1 = t.y0 + 1;
  t.wnw = ((float)x1 - t.ix) * ((float)y1 - t.iy);
  t.wne = (t.ix - (float)t.x0) * ((float)y1 - t.iy);
  t.wsw = ((float)x1 - t.ix) * (t.iy - (float)t.y0);
  t.wse = (t.ix - (float)t.x0) * (t.iy - (float)t.y0);
  t.vx0 = t.x0 >= 0 && t.x0 < w;
  t.vx1 = x1 >= 0 && x1 < w;
  t.vy0 = t.y0 >= 0 && t.y0 < h;
  t.vy1 = y1 >= 0 && y1 < h;
  return t;
}

// one image plane (h*w floats) as a buffer resource: loads at an offset past its end return 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t warp_plane(const float* im, long long hw) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)im, 0, (int)(hw * 4), 0x00020000);
}

// the four corner values, zero where the corner lies outside the image: an invalid corner
// gets an out-of-range buffer offset, so the hardware returns 0 and all four loads issue
// unconditionally, back to back (a zero corner adds +0, exactly as the skipped term would)
__device__ __forceinline__ void warp_corners(__amdgpu_buffer_rsrc_t im, const WarpTap& t, int w, float& a, float& b,
                                             float& c, float& d) {
  constexpr unsigned kOut = 0x80000000u;
  const unsigned r0 = (unsigned)(t.y0 * w), r1 = (unsigned)((t.y0 + 1) * w);
  const unsigned oa = (t.vy0 && t.vx0) ? (r0 + t.x0) * 4u : kOut;
  const unsigned ob = (t.vy0 && t.vx1) ? (r0 + t.x0 + 1) * 4u : kOut;
  const unsigned oc = (t.vy1 && t.vx0) ? (r1 + t.x0) * 4u : kOut;
  const unsigned od = (t.vy1 && t.vx1) ? (r1 + t.x0 + 1) * 4u : kOut;
  a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, oa, 0, 0));
  b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, ob, 0, 0));
  c = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, oc, 0, 0));
  d = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, od, 0, 0));
}

__device__ __forceinline__ float warp_sample(__amdgpu_buffer_rsrc_t im, const WarpTap& t, int w) {
  float a, b, c, d;
  warp_corners(im, t, w, a, b, c, d);
  float v = 0.f;
  v += a * t.wnw;
  v += b * t.wne;
  v += c * t.wsw;
  v += d * t.wse;
  return v;
}

// A wave covers 256 consecutive pixels of one row, 4 per lane 64 apart: each gather
// instruction then reads the sources of 64 consecutive output pixels (a few cache lines for
// a smooth flow), and the flow loads and output stores are 256-byte coalesced runs.
__global__ __launch_bounds__(256) void warp_fwd_kernel(const dvie_warp_desc p) {
  const int segs = (p.w + 255) >> 8;
  const long long hw = (long long)p.h * p.w;
  const int waves = p.n * p.h * segs;  // < 2^31 (checked at launch)
  const int lane = threadIdx.x & 63;
  // wave-uniform row/segment (readfirstlane), so the plane buffer resources are scalar
  for (int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * 4) {
    const int sg = wv % segs;
    const int r = wv / segs;
    const int y = r % p.h, n = r / p.h;
    WarpTap t[4];
    bool live[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = (sg << 8) + lane + 64 * k;
      live[k] = x < p.w;
      const int xl = live[k] ? x : p.w - 1;  // clamped: the loads stay unconditional
      const long long fo = (long long)y * p.w + xl;
      t[k] = warp_tap(xl, y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo], p.w, p.h,
                      p.align_corners);
    }
    for (int c = 0; c < p.c; ++c) {
      const long long plane = ((long long)n * p.c + c) * hw;
      const __amdgpu_buffer_rsrc_t im = warp_plane(p.img + plane, hw), out = warp_plane(p.out + plane, hw);
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = warp_sample(im, t[k], p.w);
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // columns past the row end: out-of-range offset, store dropped
        const unsigned off = live[k] ? (unsigned)(y * p.w + (sg << 8) + lane + 64 * k) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[k]), out, off, 0, 0);
      }
    }
  }
}

// ---- backward ----
// d/d(img) of one bilinear corner, and the flow-gradient terms, per channel (order of the
// reference autograd: corners nw, ne, sw, se)
template <typename Scatter>
__device__ __forceinline__ void warp_bwd_pixel(float a, float b, float c, float d, float go, const WarpTap& t,
                                               float& gix, float& giy, Scatter&& scatter) {
  const int x1 = t.x0 + 1, y1 = t.y0 + 1;
  // invalid corners contribute exact zeros to the flow terms (their value is 0)
  gix -= a * ((float)y1 - t.iy) * go;
  giy -= a * ((float)x1 - t.ix) * go;
  gix += b * ((float)y1 - t.iy) * go;
  giy -= b * (t.ix - (float)t.x0) * go;
  gix -= c * (t.iy - (float)t.y0) * go;
  giy += c * ((float)x1 - t.ix) * go;
  gix += d * (t.iy - (float)t.y0) * go;
  giy += d * (t.ix - (float)t.x0) * go;
  if (t.vy0 && t.vx0) scatter(t.y0, t.x0, t.wnw * go);
  if (t.vy0 && t.vx1) scatter(t.y0, x1, t.wne * go);
  if (t.vy1 && t.vx0) scatter(y1, t.x0, t.wsw * go);
  if (t.vy1 && t.vx1) scatter(y1, x1, t.wse * go);
}

__device__ __forceinline__ void warp_store_dflow(const dvie_warp_desc& p, int n, long long fo, float gix, float giy) {
  const long long hw = (long long)p.h * p.w;
  const float sx = p.align_corners ? (float)(p.w - 1) / 2.f : (float)p.w / 2.f;
  const float sy = p.align_corners ? (float)(p.h - 1) / 2.f : (float)p.h / 2.f;
  p.dflow[((long long)n * 2 + 0) * hw + fo] = -gix * sx;
  p.dflow[((long long)n * 2 + 1) * hw + fo] = -giy * sy;
}

// Image gradient by gathering instead of scattering (LDS float atomics measured at ~100
// cycles per wave instruction on gfx950, global ones at ~100 G lanes/s: both far below HBM).
// A dimg pixel c receives the bilinear weight of every sample s (output pixel) that has c as
// a corner.  Under a smooth flow those samples sit next to s*(c) = c - d(c), d(c) being the
// integer source displacement (x0 - x, y0 - y) of the sample AT c.  warp_bwd_pull_kernel
// visits the 4x4 candidates s*(c) + [-2, 1]^2 for every c and STORES dimg (no zero-fill, no
// atomics, a fixed summation order); warp_bwd_flow_kernel computes dflow and adds, with a
// global atomic, each (s, c) pair the candidate rule misses (folding / discontinuous flow).
constexpr int WP_LO = -2, WP_HI = 1;

// s*(c): c minus the integer displacement of the sample at c
__device__ __forceinline__ int2 warp_pull_origin(const dvie_warp_desc& p, const float* fl0, const float* fl1, int cx,
                                                 int cy) {
  const long long fo = (long long)cy * p.w + cx;
  const WarpTap t = warp_tap(cx, cy, fl0[fo], fl1[fo], p.w, p.h, p.align_corners);
  return make_int2(2 * cx - t.x0, 2 * cy - t.y0);
}

// the one ownership rule both passes apply: is sample (sx, sy) a candidate of cell c?
__device__ __forceinline__ bool warp_pulled(int2 o, int sx, int sy) {
  return (unsigned)(sx - o.x - WP_LO) <= (unsigned)(WP_HI - WP_LO) &&
         (unsigned)(sy - o.y - WP_LO) <= (unsigned)(WP_HI - WP_LO);
}

// a wave covers 256 consecutive dimg pixels of one row (4 per lane, 64 apart)
__global__ __launch_bounds__(256) void warp_bwd_pull_kernel(const dvie_warp_desc p) {
  const int segs = (p.w + 255) >> 8;
  const int waves = p.n * p.h * segs;
  const int lane = threadIdx.x & 63;
  const long long hw = (long long)p.h * p.w;
  for (int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * 4) {
    const int sg = wv % segs;
    const int r = wv / segs;
    const int cy = r % p.h, n = r / p.h;
    const float* fl0 = p.flow + (long long)n * 2 * hw;
    const float* fl1 = fl0 + hw;
    const __amdgpu_buffer_rsrc_t rf0 = warp_plane(fl0, hw), rf1 = warp_plane(fl1, hw);
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const int cx = (sg << 8) + lane + 64 * k;
      if (cx >= p.w) continue;
      const int2 o = warp_pull_origin(p, fl0, fl1, cx, cy);
      // phase 1: the 16 candidates' weights for c (0 where c is not one of their corners).
      // Buffer loads with 32-bit offsets; a candidate outside the image gets an out-of-range
      // offset (loads return 0) and a zero weight, so every load issues unconditionally.
      constexpr int NC = (WP_HI - WP_LO + 1) * (WP_HI - WP_LO + 1);
      unsigned off[NC];
      float fxs[NC], fys[NC];
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int sx = o.x + WP_LO + q % (WP_HI - WP_LO + 1), sy = o.y + WP_LO + q / (WP_HI - WP_LO + 1);
        const bool in = (unsigned)sx < (unsigned)p.w && (unsigned)sy < (unsigned)p.h;
        off[q] = in ? (unsigned)(sy * p.w + sx) * 4u : 0x80000000u;
        fxs[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rf0, off[q], 0, 0));
        fys[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rf1, off[q], 0, 0));
      }
      float wq[NC];
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int sx = o.x + WP_LO + q % (WP_HI - WP_LO + 1), sy = o.y + WP_LO + q / (WP_HI - WP_LO + 1);
        const float ix = unnorm(linspace_pm1(sx, p.w) - fxs[q], p.w, p.align_corners);
        const float iy = unnorm(linspace_pm1(sy, p.h) - fys[q], p.h, p.align_corners);
        const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
        const int qx = cx - x0, qy = cy - y0;  // 0/1: c is the x0/x1, y0/y1 corner of s
        // the bilinear weight exactly as warp_tap forms it (wnw / wne / wsw / wse)
        const float w = (qx == 0 ? (float)(x0 + 1) - ix : ix - (float)x0) *
                        (qy == 0 ? (float)(y0 + 1) - iy : iy - (float)y0);
        wq[q] = (off[q] != 0x80000000u && (unsigned)qx <= 1u && (unsigned)qy <= 1u) ? w : 0.f;
      }
      // phase 2: dimg[c] = sum over candidates of weight * dout[s], in candidate order
      // (a zero weight adds +0: the candidate did not hit c)
      for (int ch = 0; ch < p.c; ++ch) {
        const long long plane = ((long long)n * p.c + ch) * hw;
        const __amdgpu_buffer_rsrc_t rg = warp_plane(p.dout + plane, hw);
        float g[NC];
#pragma unroll
        for (int q = 0; q < NC; ++q) g[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, off[q], 0, 0));
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NC; ++q) acc += wq[q] * g[q];
        p.dimg[plane + (long long)cy * p.w + cx] = acc;
      }
    }
  }
}

// dflow for every sample and, with dimg, the (sample, corner) pairs the pull pass misses
// (global atomics, launched after it).  A wave covers 256 consecutive pixels of a row (4 per
// lane, 64 apart), so the image planes are wave-uniform buffer resources.
__global__ __launch_bounds__(256) void warp_bwd_flow_kernel(const dvie_warp_desc p) {
  const int segs = (p.w + 255) >> 8;
  const int waves = p.n * p.h * segs;
  const int lane = threadIdx.x & 63;
  const long long hw = (long long)p.h * p.w;
  for (int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * 4) {
    const int sg = wv % segs;
    const int r = wv / segs;
    const int y = r % p.h, n = r / p.h;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const int x = (sg << 8) + lane + 64 * k;
      const bool live = x < p.w;
      const int xl = live ? x : p.w - 1;
      const long long fo = (long long)y * p.w + xl;
      const WarpTap t = warp_tap(xl, y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo],
                                 p.w, p.h, p.align_corners);
      // (sample, corner) pairs the pull pass misses (evaluated once, shared by all channels)
      bool far[4] = {false, false, false, false};
      if (p.dimg && live) {
        const float* fl0 = p.flow + (long long)n * 2 * hw;
        const int cxs[4] = {t.x0, t.x0 + 1, t.x0, t.x0 + 1}, cys[4] = {t.y0, t.y0, t.y0 + 1, t.y0 + 1};
        const bool val[4] = {t.vy0 && t.vx0, t.vy0 && t.vx1, t.vy1 && t.vx0, t.vy1 && t.vx1};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (val[q]) far[q] = !warp_pulled(warp_pull_origin(p, fl0, fl0 + hw, cxs[q], cys[q]), xl, y);
      }
      const bool any_far = far[0] || far[1] || far[2] || far[3];
      float gix = 0.f, giy = 0.f;
      for (int c = 0; c < p.c; ++c) {
        const long long base = ((long long)n * p.c + c) * hw;
        float a, b, cc, dd;
        warp_corners(warp_plane(p.img + base, hw), t, p.w, a, b, cc, dd);
        const float go = p.dout[base + fo];
        warp_bwd_pixel(a, b, cc, dd, go, t, gix, giy, [](int, int, float) {});
        if (any_far) {
          if (far[0]) atomicAdd(p.dimg + base + (long long)t.y0 * p.w + t.x0, t.wnw * go);
          if (far[1]) atomicAdd(p.dimg + base + (long long)t.y0 * p.w + t.x0 + 1, t.wne * go);
          if (far[2]) atomicAdd(p.dimg + base + (long long)(t.y0 + 1) * p.w + t.x0, t.wsw * go);
          if (far[3]) atomicAdd(p.dimg + base + (long long)(t.y0 + 1) * p.w + t.x0 + 1, t.wse * go);
        }
      }
      if (p.dflow && live) warp_store_dflow(p, n, fo, gix, giy);
    }
  }
}

__global__ void adamax_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                              float* __restrict__ u, long long n, float clr, float b1, float b2, float eps,
                              float wd, const float* __restrict__ stepp, double lr, double b1d) {
  // device-resident step count (graph-captured steps): clr = lr / (1 - b1^t) in double
  // from the caller's double lr / beta1, exactly as the host computes it for an eager step
  if (stepp) clr = (float)(lr / (1.0 - pow(b1d, (double)stepp[0])));
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float gr = g[i];
    const float pv = p[i];
    if (wd != 0.f) gr += wd * pv;
    // torch lerp: weight < 0.5 -> self + w*(end-self)
    const float w = 1.f - b1;
    const float mv = m[i];
    const float mn = (w < 0.5f) ? mv + w * (gr - mv) : gr - (gr - mv) * (1.f - w);
    const float un = fmaxf(u[i] * b2, fabsf(gr) + eps);
    m[i] = mn;
    u[i] = un;
    p[i] = pv - clr * (mn / un);
  }
}

// one-element increment of a device step counter (thread-indexed: a vector store)
__global__ void step_inc_kernel(float* step) {
  if (threadIdx.x == 0) step[threadIdx.x] += 1.f;
}

__global__ void scale_kernel(float* p, long long n, float s) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] *= s;
}

static int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace dvie

using namespace dvie;

extern "C" {

int dvie_warp_fwd(const dvie_warp_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->flow && d->out && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "warp: args");
  const long long waves = (long long)d->n * d->h * ((d->w + 255) / 256);
  DVIE_CHECK_ARG(waves < (1LL << 31) && (long long)d->h * d->w < (1LL << 29), "warp: size");
  hipLaunchKernelGGL(warp_fwd_kernel, dim3(grid_for(waves * 256)), dim3(256), 0, (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}


size_t dvie_warp_ws_floats(const dvie_warp_desc* d) {
  (void)d;
  return 0;  // the backward needs no workspace (kept for ABI stability)
}

int dvie_warp_bwd(const dvie_warp_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->flow && d->dout && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "warp: args");
  DVIE_CHECK_ARG((long long)d->h * d->w < (1LL << 29), "warp: size");
  hipStream_t s = (hipStream_t)stream;
  const long long waves = (long long)d->n * d->h * ((d->w + 255) / 256);
  DVIE_CHECK_ARG(waves < (1LL << 31), "warp: size");
  if (d->dimg) hipLaunchKernelGGL(warp_bwd_pull_kernel, dim3(grid_for(waves * 256)), dim3(256), 0, s, *d);
  hipLaunchKernelGGL(warp_bwd_flow_kernel, dim3(grid_for(waves * 256)), dim3(256), 0, s, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_adamax(float* p, const float* g, float* m, float* u, long long n, float clr, float b1, float b2, float eps,
                float wd, void* stream) {
  DVIE_CHECK_ARG(p && g && m && u && n >= 0, "adamax: args");
  if (n == 0) return DVIE_OK;
  hipLaunchKernelGGL(adamax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, u, n, clr, b1, b2,
                     eps, wd, (const float*)nullptr, 0.0, 0.0);
  DVIE_RETURN_LAUNCH();
}

int dvie_adamax_dev(float* p, const float* g, float* m, float* u, long long n, double lr, double b1, double b2,
                    double eps, double wd, const float* step, void* stream) {
  DVIE_CHECK_ARG(p && g && m && u && step && n >= 0, "adamax_dev: args");
  if (n == 0) return DVIE_OK;
  hipLaunchKernelGGL(adamax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, u, n, 0.f,
                     (float)b1, (float)b2, (float)eps, (float)wd, step, lr, b1);
  DVIE_RETURN_LAUNCH();
}

int dvie_step_inc(float* step, void* stream) {
  DVIE_CHECK_ARG(step, "step_inc: null");
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step);
  DVIE_RETURN_LAUNCH();
}

int dvie_scale(float* p, long long n, float s, void* stream) {
  DVIE_CHECK_ARG(p && n >= 0, "scale: args");
  if (n == 0) return DVIE_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, n, s);
  DVIE_RETURN_LAUNCH();
}

int dvie_run_ops(const dvie_op* ops, int n, void* stream) {
  for (int i = 0; i < n; ++i) {
    int rc = DVIE_OK;
    const dvie_op& o = ops[i];
    switch (o.kind) {
      case DVIE_OP_CONV: rc = dvie_conv2d_fwd(&o.u.conv, stream); break;
      case DVIE_OP_WGRAD: rc = dvie_conv2d_wgrad(&o.u.wgrad, stream); break;
      case DVIE_OP_WREDUCE: rc = dvie_wgrad_reduce(&o.u.wreduce, stream); break;
      case DVIE_OP_COLSUM: rc = dvie_colsum(&o.u.colsum, stream); break;
      case DVIE_OP_EW: rc = dvie_ew(&o.u.ew, stream); break;
      case DVIE_OP_LOSS: rc = dvie_loss(&o.u.loss, stream); break;
      case DVIE_OP_PACK: rc = dvie_pack_weights(o.u.pack.descs_dev, o.u.pack.n, o.u.pack.max_elems, stream); break;
      case DVIE_OP_BN_FWD: rc = dvie_bn_fwd(&o.u.bn, stream); break;
      case DVIE_OP_BN_BWD: rc = dvie_bn_bwd(&o.u.bn, stream); break;
      case DVIE_OP_HEAD_FWD: rc = dvie_head_fwd(&o.u.head, stream); break;
      case DVIE_OP_HEAD_BWD: rc = dvie_head_bwd(&o.u.head, stream); break;
      case DVIE_OP_ATTN: rc = dvie_attn(&o.u.attn, stream); break;
      default: set_error("run_ops: unknown op kind %d at %d", o.kind, i); return DVIE_EINVAL;
    }
    if (rc != DVIE_OK) {
      if (rc == DVIE_EINVAL) {
        // keep the message, prefix the op index
        char buf[512];
        snprintf(buf, sizeof(buf), "op %d (kind %d): %s", i, o.kind, dvie_last_error());
        set_error("%s", buf);
      }
      return rc;
    }
  }
  return DVIE_OK;
}

size_t dvie_abi_sizeof(int which) {
  switch (which) {
    case 0: return sizeof(dvie_op);
    case DVIE_OP_CONV: return sizeof(dvie_conv_desc);
    case DVIE_OP_WGRAD: return sizeof(dvie_wgrad_desc);
    case DVIE_OP_WREDUCE: return sizeof(dvie_wreduce_desc);
    case DVIE_OP_COLSUM: return sizeof(dvie_colsum_desc);
    case DVIE_OP_EW: return sizeof(dvie_ew_desc);
    case DVIE_OP_LOSS: return sizeof(dvie_loss_desc);
    case DVIE_OP_PACK: return sizeof(dvie_pack_desc);
    case DVIE_OP_BN_FWD: return sizeof(dvie_bn_desc);
    case DVIE_OP_HEAD_FWD: return sizeof(dvie_head_desc);
    case DVIE_OP_ATTN: return sizeof(dvie_attn_desc);
    case 100: return sizeof(dvie_warp_desc);
    case 101: return sizeof(dvie_softmax_desc);
    case 102: return sizeof(dvie_sn_layer);
    case 103: return sizeof(dvie_clip_desc);
    default: return 0;
  }
}

const char* dvie_version(void) { return "dvie 0.1.0 gfx950"; }

}  // extern "C"
