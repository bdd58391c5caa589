// Bilinear flow warp (grid_sample, zeros padding) forward/backward, the fused Adamax
// step over a flat parameter buffer, and the op-list executor / ABI helpers.
//
// Reference: FlowWrapper utils/net_utils.py:89-114 (warp / warp_back l.116-129);
// torch.optim.Adamax at runners/InterTrainer.py:79.
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace dvie {

// torch.linspace(-1, 1, n)[i] as computed by the CPU kernel (two-sided)
__device__ __forceinline__ float linspace_pm1(int i, int n) {
  if (n <= 1) return -1.f;
  const float step = 2.f / (float)(n - 1);
  // one rounding per half, as torch.linspace's CPU kernel (bit-equal at every size checked)
  return (i < n / 2) ? __builtin_fmaf(step, (float)i, -1.f) : __builtin_fmaf(-step, (float)(n - 1 - i), 1.f);
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
// gets an out-of-range buffer offset, so the hardware returns 0 (a zero corner adds +0,
// exactly as the skipped term would)
// pair = (wave-uniform) every lane's two columns lie inside the image
__device__ __forceinline__ void warp_corners(__amdgpu_buffer_rsrc_t im, const WarpTap& t, int w, float& a, float& b,
                                             float& c, float& d, bool pair = false) {
  constexpr unsigned kOut = 0x80000000u;
  const unsigned r0 = (unsigned)(t.y0 * w), r1 = (unsigned)((t.y0 + 1) * w);
  if (pair) {
    // one 8-byte load per corner row (the vector-memory pipe, not the bytes, bounds these
    // gathers: one instruction per row instead of two)
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(im, t.vy0 ? (r0 + t.x0) * 4u : kOut, 0, 0);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(im, t.vy1 ? (r1 + t.x0) * 4u : kOut, 0, 0);
    a = __uint_as_float(u[0]);
    b = __uint_as_float(u[1]);
    c = __uint_as_float(v[0]);
    d = __uint_as_float(v[1]);
    return;
  }
  const unsigned oa = (t.vy0 && t.vx0) ? (r0 + t.x0) * 4u : kOut;
  const unsigned ob = (t.vy0 && t.vx1) ? (r0 + t.x0 + 1) * 4u : kOut;
  const unsigned oc = (t.vy1 && t.vx0) ? (r1 + t.x0) * 4u : kOut;
  const unsigned od = (t.vy1 && t.vx1) ? (r1 + t.x0 + 1) * 4u : kOut;
  a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, oa, 0, 0));
  b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, ob, 0, 0));
  c = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, oc, 0, 0));
  d = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(im, od, 0, 0));
}

__device__ __forceinline__ float warp_blend(float a, float b, float c, float d, const WarpTap& t) {
  float v = 0.f;
  v += a * t.wnw;
  v += b * t.wne;
  v += c * t.wsw;
  v += d * t.wse;
  return v;
}

// These kernels are latency-bound gathers: a wave's time is its chain of dependent memory
// round trips, not its bytes.  So each kernel issues every load it can before the first use
// -- all channels of all its pixels at once (CC = the channel count as a compile-time
// constant; CC = 0 is the generic per-channel loop) -- and stores only after the loads.
//
// Forward: a wave covers 256 consecutive pixels of one row, 4 per lane 64 apart: each gather
// instruction reads the sources of 64 consecutive output pixels (a few cache lines for a
// smooth flow), and the flow loads and output stores are 256-byte coalesced runs.
//
// xcd: workgroups are dealt to the 8 XCDs round-robin by index; with xcd set (and a grid that
// is a multiple of 8) workgroup b takes the job slot (b % 8) * (grid / 8) + b / 8, so each XCD
// walks a contiguous band of rows and the source rows two neighbouring output rows share are
// gathered into one L2 instead of two.
template <int CC, int LAUX = 0, int SAUX = 0, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void warp_fwd_kernel(const dvie_warp_desc p, int xcd) {
  const int segs = (p.w + 255) >> 8;
  const long long hw = (long long)p.h * p.w;
  const int waves = p.n * p.h * segs;  // < 2^31 (checked at launch)
  const int lane = threadIdx.x & 63;
  const int g = gridDim.x;
  const int vb = (xcd && (g & 7) == 0) ? (int)(blockIdx.x & 7) * (g >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  // wave-uniform row/segment (readfirstlane), so the plane buffer resources are scalar
  for (int wv = __builtin_amdgcn_readfirstlane(vb * WPB + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * WPB) {
    const int sg = wv % segs;
    const int r = wv / segs;
    const int y = r % p.h, n = r / p.h;
    const __amdgpu_buffer_rsrc_t rf0 = warp_plane(p.flow + (long long)n * 2 * hw, hw);
    const __amdgpu_buffer_rsrc_t rf1 = warp_plane(p.flow + ((long long)n * 2 + 1) * hw, hw);
    float fx[4], fy[4];
    bool live[4], pair[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = (sg << 8) + lane + 64 * k;
      live[k] = x < p.w;
      const unsigned fo = (unsigned)(y * p.w + (live[k] ? x : p.w - 1)) * 4u;  // clamped: loads stay unconditional
      fx[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rf0, fo, 0, LAUX));
      fy[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rf1, fo, 0, LAUX));
    }
    WarpTap t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = (sg << 8) + lane + 64 * k;
      t[k] = warp_tap(live[k] ? x : p.w - 1, y, fx[k], fy[k], p.w, p.h, p.align_corners);
      pair[k] = __all(t[k].vx0 && t[k].vx1);
    }
    auto store = [&](int c, const float* o) {
      const __amdgpu_buffer_rsrc_t out = warp_plane(p.out + ((long long)n * p.c + c) * hw, hw);
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // columns past the row end: out-of-range offset, store dropped
        const unsigned off = live[k] ? (unsigned)(y * p.w + (sg << 8) + lane + 64 * k) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[k]), out, off, 0, SAUX);
      }
    };
    if constexpr (CC > 0) {
      float v[CC][4][4];
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        const __amdgpu_buffer_rsrc_t im = warp_plane(p.img + ((long long)n * CC + c) * hw, hw);
#pragma unroll
        for (int k = 0; k < 4; ++k) warp_corners(im, t[k], p.w, v[c][k][0], v[c][k][1], v[c][k][2], v[c][k][3], pair[k]);
      }
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = warp_blend(v[c][k][0], v[c][k][1], v[c][k][2], v[c][k][3], t[k]);
        store(c, o);
      }
    } else {
      for (int c = 0; c < p.c; ++c) {
        const __amdgpu_buffer_rsrc_t im = warp_plane(p.img + ((long long)n * p.c + c) * hw, hw);
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float a, b, cc, d;
          warp_corners(im, t[k], p.w, a, b, cc, d, pair[k]);
          o[k] = warp_blend(a, b, cc, d, t[k]);
        }
        store(c, o);
      }
    }
  }
}

// ---- backward ----
// the flow-gradient terms of one channel (order of the reference autograd: corners nw, ne,
// sw, se); invalid corners contribute exact zeros (their value is 0)
__device__ __forceinline__ void warp_dflow_terms(float a, float b, float c, float d, float go, const WarpTap& t,
                                                 float& gix, float& giy) {
  const int x1 = t.x0 + 1, y1 = t.y0 + 1;
  gix -= a * ((float)y1 - t.iy) * go;
  giy -= a * ((float)x1 - t.ix) * go;
  gix += b * ((float)y1 - t.iy) * go;
  giy -= b * (t.ix - (float)t.x0) * go;
  gix -= c * (t.iy - (float)t.y0) * go;
  giy += c * ((float)x1 - t.ix) * go;
  gix += d * (t.iy - (float)t.y0) * go;
  giy += d * (t.ix - (float)t.x0) * go;
}

// Image gradient by gathering instead of scattering (LDS float atomics measured at ~100
// cycles per wave instruction on gfx950, global ones at ~100 G lanes/s: both far below HBM).
// A dimg pixel c receives the bilinear weight of every sample s (output pixel) that has c as
// a corner: x0(s) in {cx - 1, cx} and y0(s) in {cy - 1, cy}.  Write x0(s) = sx + D(s), D the
// integer part of the sample's displacement; where D(s) = D(c) the samples are
// sx in {o.x - 1, o.x}, o = 2c - (x0, y0)(c).  The pull window of c, per axis, is
//   WIN = 4: o.x + {-2 .. 1}: every sample with |delta(s) - delta(c)| < 1 px;
//   WIN = 3: the side the fractional part f(c) = ix(c) - x0(c) points to, o.x + {-1 .. 1}
//            for f < 1/2 (D(s) in {D - 1, D}), o.x + {-2 .. 0} otherwise: every sample with
//            |delta(s) - delta(c)| < 1/2 px.
// Samples a window misses (folding / discontinuous flow) are added with atomics.
//
// Three launches (one pixel per lane, a wave = 64 consecutive pixels of a row):
//   tap   per sample: (ix, iy) into the workspace (8 B, exact fp32: every later weight is
//         formed from them exactly as warp_tap does) and dflow.
//   pull  per dimg pixel: the window candidates' weights from their stored taps, dimg as a
//         plain store (no zero-fill, no atomics, a fixed summation order); and per sample
//         (the same index) the ownership check of its 4 corners -> a far-corner byte.
//   far   reads the far bytes (four per lane) and adds the far corners with global atomics.
// Workspace (dvie_warp_ws_floats): taps 2*n*h*w floats, then n*h*w far bytes.
constexpr unsigned kWarpOOB = 0x80000000u;

struct PullWin {
  int sx0, sy0;  // first column / row of the window of samples pulled by c
};

// c's window, from the stored tap (ix, iy) of the sample AT c
template <int WIN>
__device__ __forceinline__ PullWin warp_win(int cx, int cy, float ix, float iy) {
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  PullWin w;
  w.sx0 = 2 * cx - (int)fx0 + (WIN == 4 ? -2 : (ix - fx0 < 0.5f ? -1 : -2));
  w.sy0 = 2 * cy - (int)fy0 + (WIN == 4 ? -2 : (iy - fy0 < 0.5f ? -1 : -2));
  return w;
}

template <int WIN>
__device__ __forceinline__ bool warp_pulled(const PullWin& w, int sx, int sy) {
  return (unsigned)(sx - w.sx0) <= (unsigned)(WIN - 1) && (unsigned)(sy - w.sy0) <= (unsigned)(WIN - 1);
}

__device__ __forceinline__ float2 warp_ld_tap(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}

__device__ __forceinline__ unsigned char* warp_far_bytes(const dvie_warp_desc& p) {
  return (unsigned char*)(p.ws + ((2LL * p.n * p.h * p.w + 3) & ~3LL));  // 16-B aligned
}

// wave -> (image, row, 64-pixel segment); lane -> column
struct WarpRow {
  int n, y, x;
};
__device__ __forceinline__ WarpRow warp_row(const dvie_warp_desc& p, int wv, int lane) {
  const int segs = (p.w + 63) >> 6;
  const int sg = wv % segs, r = wv / segs;
  WarpRow q;
  q.y = r % p.h;
  q.n = r / p.h;
  q.x = (sg << 6) + lane;
  return q;
}

// tap pass
template <int CC>
__global__ __launch_bounds__(256) void warp_bwd_tap_kernel(const dvie_warp_desc p) {
  const int waves = p.n * p.h * ((p.w + 63) >> 6);
  const int lane = threadIdx.x & 63;
  const long long hw = (long long)p.h * p.w;
  for (int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * 4) {
    const WarpRow q = warp_row(p, wv, lane);
    if (q.x >= p.w) continue;
    const int n = q.n;
    const long long fo = (long long)q.y * p.w + q.x;
    const WarpTap t = warp_tap(q.x, q.y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo],
                               p.w, p.h, p.align_corners);
    if (p.dflow) {
      const bool pair = __all(t.vx0 && t.vx1);
      float gix = 0.f, giy = 0.f;
      if constexpr (CC > 0) {
        float v[CC][4], go[CC];
#pragma unroll
        for (int c = 0; c < CC; ++c) {
          const long long base = ((long long)n * CC + c) * hw;
          warp_corners(warp_plane(p.img + base, hw), t, p.w, v[c][0], v[c][1], v[c][2], v[c][3], pair);
          go[c] = p.dout[base + fo];
        }
#pragma unroll
        for (int c = 0; c < CC; ++c) warp_dflow_terms(v[c][0], v[c][1], v[c][2], v[c][3], go[c], t, gix, giy);
      } else {
        for (int c = 0; c < p.c; ++c) {
          const long long base = ((long long)n * p.c + c) * hw;
          float a, b, cc, dd;
          warp_corners(warp_plane(p.img + base, hw), t, p.w, a, b, cc, dd, pair);
          warp_dflow_terms(a, b, cc, dd, p.dout[base + fo], t, gix, giy);
        }
      }
      const float sx = p.align_corners ? (float)(p.w - 1) / 2.f : (float)p.w / 2.f;
      const float sy = p.align_corners ? (float)(p.h - 1) / 2.f : (float)p.h / 2.f;
      p.dflow[((long long)n * 2 + 0) * hw + fo] = -gix * sx;
      p.dflow[((long long)n * 2 + 1) * hw + fo] = -giy * sy;
    }
    if (p.dimg) *(float2*)(p.ws + 2 * ((long long)n * hw + fo)) = make_float2(t.ix, t.iy);
  }
}

// pull pass
template <int WIN, int CC>
__global__ __launch_bounds__(256) void warp_bwd_pull_kernel(const dvie_warp_desc p) {
  constexpr int NC = WIN * WIN;
  const int waves = p.n * p.h * ((p.w + 63) >> 6);
  const int lane = threadIdx.x & 63;
  const long long hw = (long long)p.h * p.w;
  for (int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); wv < waves;
       wv += gridDim.x * 4) {
    const WarpRow rq = warp_row(p, wv, lane);
    const int n = rq.n, cx = rq.x, cy = rq.y;
    if (cx >= p.w) continue;
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc(p.ws + 2 * (long long)n * hw, 0, (int)(hw * 8), 0x00020000);
    const float2 tc = warp_ld_tap(rt, (unsigned)(cy * p.w + cx) * 8u);
    // round trip 2: the candidates' taps, their dout values (every channel), and the taps of
    // the corners of the sample AT c (for the ownership check), all issued together
    const int x0 = (int)floorf(tc.x), y0 = (int)floorf(tc.y);
    const PullWin win = warp_win<WIN>(cx, cy, tc.x, tc.y);
    // candidate offsets: the window's rows and columns are checked once (separable)
    int rowo[WIN];
    bool rowok[WIN], colok[WIN];
#pragma unroll
    for (int j = 0; j < WIN; ++j) {
      rowok[j] = (unsigned)(win.sy0 + j) < (unsigned)p.h;
      colok[j] = (unsigned)(win.sx0 + j) < (unsigned)p.w;
      rowo[j] = (win.sy0 + j) * p.w + win.sx0;
    }
    unsigned off[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q)
      off[q] = rowok[q / WIN] && colok[q % WIN] ? (unsigned)(rowo[q / WIN] + q % WIN) : kWarpOOB;
    // wide: every lane's window columns lie inside the image (wave-uniform), so a window row
    // is one contiguous run -- its taps one 16-B + one 8-B (WIN 3) or two 16-B loads, its
    // dout values one 12-B / 16-B load per channel -- instead of one load per candidate
    // (these gathers are bound by vector-memory instructions, not bytes)
    const bool wide = __all(colok[0] && colok[WIN - 1]);
    float2 tq[NC];
    if (wide) {
#pragma unroll
      for (int j = 0; j < WIN; ++j) {
        const unsigned rb = rowok[j] ? (unsigned)rowo[j] * 8u : kWarpOOB;
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rt, rb, 0, 0);
        tq[j * WIN] = make_float2(__uint_as_float(a[0]), __uint_as_float(a[1]));
        tq[j * WIN + 1] = make_float2(__uint_as_float(a[2]), __uint_as_float(a[3]));
        if constexpr (WIN == 3) {
          tq[j * WIN + 2] = warp_ld_tap(rt, rowok[j] ? rb + 16u : kWarpOOB);
        } else {
          const auto b = __builtin_amdgcn_raw_buffer_load_b128(rt, rowok[j] ? rb + 16u : kWarpOOB, 0, 0);
          tq[j * WIN + 2] = make_float2(__uint_as_float(b[0]), __uint_as_float(b[1]));
          tq[j * WIN + 3] = make_float2(__uint_as_float(b[2]), __uint_as_float(b[3]));
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < NC; ++q) tq[q] = warp_ld_tap(rt, off[q] == kWarpOOB ? kWarpOOB : off[q] * 8u);
    }
    auto load_go = [&](int ch, float* g) {
      const __amdgpu_buffer_rsrc_t rg = warp_plane(p.dout + ((long long)n * p.c + ch) * hw, hw);
      if (wide) {
#pragma unroll
        for (int j = 0; j < WIN; ++j) {
          const unsigned rb = rowok[j] ? (unsigned)rowo[j] * 4u : kWarpOOB;
          if constexpr (WIN == 3) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(rg, rb, 0, 0);
#pragma unroll
            for (int i = 0; i < 3; ++i) g[j * WIN + i] = __uint_as_float(v[i]);
          } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rg, rb, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) g[j * WIN + i] = __uint_as_float(v[i]);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < NC; ++q)
          g[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               rg, off[q] == kWarpOOB ? kWarpOOB : off[q] * 4u, 0, 0));
      }
    };
    float gv[CC > 0 ? CC : 1][NC];
    if constexpr (CC > 0) {
#pragma unroll
      for (int ch = 0; ch < CC; ++ch) load_go(ch, gv[ch]);
    }
    // the corners' taps: the two of a corner row are adjacent (one 16-B load when every
    // lane's x0 and x0 + 1 lie inside the image)
    float2 te[4];
    bool ve[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) ve[q] = (unsigned)(x0 + (q & 1)) < (unsigned)p.w && (unsigned)(y0 + (q >> 1)) < (unsigned)p.h;
    if (__all(x0 >= 0 && x0 + 1 < p.w)) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rt, ve[2 * r] ? (unsigned)((y0 + r) * p.w + x0) * 8u : kWarpOOB, 0, 0);
        te[2 * r] = make_float2(__uint_as_float(a[0]), __uint_as_float(a[1]));
        te[2 * r + 1] = make_float2(__uint_as_float(a[2]), __uint_as_float(a[3]));
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        te[q] = warp_ld_tap(rt, ve[q] ? (unsigned)((y0 + (q >> 1)) * p.w + x0 + (q & 1)) * 8u : kWarpOOB);
    }
    // the candidates' weights for c (0 where c is not one of their corners, or the candidate
    // lies outside the image).  c is the x0 corner of s iff cx <= ix < cx + 1 and the x1
    // corner iff cx - 1 <= ix < cx, so the factor warp_tap forms, (x0 + 1) - ix or ix - x0,
    // is (cx + 1) - ix or ix - (cx - 1): the same fp32 operations, without floor/convert
    const float fcx = (float)cx, fcy = (float)cy;
    const float cxp = fcx + 1.f, cxm = fcx - 1.f, cyp = fcy + 1.f, cym = fcy - 1.f;
    float wq[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const float ix = tq[q].x, iy = tq[q].y;
      const float wx = ix >= fcx ? cxp - ix : ix - cxm;
      const float wy = iy >= fcy ? cyp - iy : iy - cym;
      const bool hit = off[q] != kWarpOOB && ix >= cxm && ix < cxp && iy >= cym && iy < cyp;
      wq[q] = hit ? wx * wy : 0.f;
    }
    // dimg[c] = sum over candidates of weight * dout[s], in candidate order (a zero weight
    // adds +0: the candidate did not hit c)
    const long long co = (long long)cy * p.w + cx;
    if constexpr (CC > 0) {
#pragma unroll
      for (int ch = 0; ch < CC; ++ch) {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NC; ++q) acc += wq[q] * gv[ch][q];
        p.dimg[((long long)n * CC + ch) * hw + co] = acc;
      }
    } else {
      for (int ch = 0; ch < p.c; ++ch) {
        load_go(ch, gv[0]);
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NC; ++q) acc += wq[q] * gv[0][q];
        p.dimg[((long long)n * p.c + ch) * hw + co] = acc;
      }
    }
    // ownership of the sample AT c (s = c): bit q set = corner q's window misses it
    unsigned fb = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ex = x0 + (q & 1), ey = y0 + (q >> 1);
      if (ve[q] && !warp_pulled<WIN>(warp_win<WIN>(ex, ey, te[q].x, te[q].y), cx, cy)) fb |= 1u << q;
    }
    warp_far_bytes(p)[(long long)n * hw + co] = (unsigned char)fb;
  }
}

// far pass: four samples per lane (one 4-byte load of far bytes); every set bit adds that
// corner with a global atomic
__device__ __forceinline__ void warp_far_sample(const dvie_warp_desc& p, long long gs, unsigned fb, long long hw) {
  const int n = (int)(gs / hw);
  const long long fo = gs - (long long)n * hw;
  // the stored tap (the weights the pull pass forms for its candidates, bit for bit)
  const float2 tp = *(const float2*)(p.ws + 2 * gs);
  const float ix = tp.x, iy = tp.y;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float wts[4] = {((fx0 + 1.f) - ix) * ((fy0 + 1.f) - iy), (ix - fx0) * ((fy0 + 1.f) - iy),
                        ((fx0 + 1.f) - ix) * (iy - fy0), (ix - fx0) * (iy - fy0)};
  for (int c = 0; c < p.c; ++c) {
    const long long base = ((long long)n * p.c + c) * hw;
    const float go = p.dout[base + fo];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (fb & (1u << q)) atomicAdd(p.dimg + base + (long long)(y0 + (q >> 1)) * p.w + x0 + (q & 1), wts[q] * go);
  }
}

__global__ __launch_bounds__(256) void warp_bwd_far_kernel(const dvie_warp_desc p) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * hw;
  const unsigned char* fbytes = warp_far_bytes(p);
  for (long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < total;
       i0 += (long long)gridDim.x * blockDim.x * 4) {
    unsigned w4;
    if (i0 + 4 <= total) {
      w4 = *(const unsigned*)(fbytes + i0);
    } else {
      w4 = 0;
      for (int j = 0; i0 + j < total; ++j) w4 |= (unsigned)fbytes[i0 + j] << (8 * j);
    }
    if (!w4) continue;
    for (int j = 0; j < 4; ++j)
      if ((w4 >> (8 * j)) & 15u) warp_far_sample(p, i0 + j, (w4 >> (8 * j)) & 15u, hw);
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
  // waves per workgroup: 8 once the frames outgrow the L2s (8x3x1024x2048: 101.5 -> 95.5 us,
  // 0.66 -> 0.70 of HBM), 4 below (8x3x256x512: 7.5 vs 8.4 us; 16 loses at both sizes:
  // profiles/r06/warp_wpb/).  DVIE_WARP_FWD_WPB (A/B, read per launch): 4 / 8 / 16
  const char* we = getenv("DVIE_WARP_FWD_WPB");
  const int wpb = we && *we ? atoi(we) : (waves >= 32768 ? 8 : 4);
  DVIE_CHECK_ARG(wpb == 4 || wpb == 8 || wpb == 16, "warp: DVIE_WARP_FWD_WPB must be 4, 8 or 16");
  // one workgroup per wpb waves (jobs) up to 8192 workgroups
  int grid = (int)((waves + wpb - 1) / wpb < 8192 ? (waves + wpb - 1) / wpb : 8192);
  if (const char* e = getenv("DVIE_WARP_FWD_GRID")) {  // A/B: blocks = min(jobs / 4, cap)
    const long long need = (waves + 3) / 4, cap = atoi(e);
    if (cap > 0) grid = (int)(need < cap ? need : cap);
  }
  // flow loads and output stores read / written once: non-temporal (aux 2).  Same box,
  // 8x3x256x512 8.2 -> 7.4 us, 8x3x1024x2048 128.9 -> 121.5 us (profiles/r04warpnt/).
  // DVIE_WARP_NT (A/B, read per launch): 0 = default policy, 1 = non-temporal stores only
  const char* nt = getenv("DVIE_WARP_NT");
  const int ntm = nt && *nt ? atoi(nt) : 2;
  // XCD bands pay off once the frames outgrow the L2s: 8x3x1024x2048 121.0 -> 100.2 us
  // (0.555 -> 0.670 of HBM), while at 8x3x256x512 (12.6 MB) they cost 7.2 -> 8.6 us
  // (profiles/r04aa/).  DVIE_WARP_XCD (A/B, read per launch): 1 = always, 0 = never
  const char* xe = getenv("DVIE_WARP_XCD");
  const int xcd = xe && *xe ? atoi(xe) : ((long long)d->n * d->c * d->h * d->w * 4 > (64ll << 20));
  if (d->c == 3 && ntm == 2 && wpb == 8)
    DVIE_LAUNCH((warp_fwd_kernel<3, 2, 2, 8>), dim3(grid), dim3(512), 0, (hipStream_t)stream, *d, xcd);
  else if (d->c == 3 && ntm == 2 && wpb == 16)
    DVIE_LAUNCH((warp_fwd_kernel<3, 2, 2, 16>), dim3(grid), dim3(1024), 0, (hipStream_t)stream, *d, xcd);
  else if (d->c == 3 && ntm == 1)
    DVIE_LAUNCH((warp_fwd_kernel<3, 0, 2>), dim3(grid), dim3(256), 0, (hipStream_t)stream, *d, xcd);
  else if (d->c == 3 && ntm == 2)
    DVIE_LAUNCH((warp_fwd_kernel<3, 2, 2>), dim3(grid), dim3(256), 0, (hipStream_t)stream, *d, xcd);
  else if (d->c == 3)
    DVIE_LAUNCH(warp_fwd_kernel<3>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *d, xcd);
  else
    DVIE_LAUNCH(warp_fwd_kernel<0>, dim3(grid), dim3(256), 0, (hipStream_t)stream, *d, xcd);
  DVIE_RETURN_LAUNCH();
}

size_t dvie_warp_ws_floats(const dvie_warp_desc* d) {
  if (!d || !d->dimg) return 0;  // dflow only: no workspace
  const size_t px = (size_t)d->n * d->h * d->w;
  return (2 * px + 3) / 4 * 4 + (px + 15) / 16 * 4;  // taps, far bytes (16-B aligned)
}

// pull window width (see warp_bwd_pull_kernel): 4 by default -- a noisy flow (a flow net early
// in training) stays off the atomic path; DVIE_WARP_WIN=3 for A/B runs (15% faster on a
// smooth flow, 22% slower with 0.2 px per-pixel noise at 1024x2048: profiles/r02_warp/)
static const int warp_win_env = getenv("DVIE_WARP_WIN") && atoi(getenv("DVIE_WARP_WIN")) == 3 ? 3 : 4;

int dvie_warp_bwd(const dvie_warp_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->flow && d->dout && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "warp: args");
  DVIE_CHECK_ARG((long long)d->h * d->w < (1LL << 28), "warp: size");  // tap offsets: 8 B/px
  DVIE_CHECK_ARG((long long)d->n * d->h * d->w < (1LL << 31), "warp: size");
  DVIE_CHECK_ARG(!d->dimg || d->ws, "warp: dimg needs the workspace (dvie_warp_ws_floats)");
  hipStream_t s = (hipStream_t)stream;
  const long long waves = (long long)d->n * d->h * ((d->w + 63) / 64);
  DVIE_CHECK_ARG(waves < (1LL << 31), "warp: size");
  if (!d->dimg && !d->dflow) return DVIE_OK;
  const int grid = (int)std::min<long long>((waves + 3) / 4, 16384);
  const bool c3 = d->c == 3;
  if (c3)
    DVIE_LAUNCH(warp_bwd_tap_kernel<3>, dim3(grid), dim3(256), 0, s, *d);
  else
    DVIE_LAUNCH(warp_bwd_tap_kernel<0>, dim3(grid), dim3(256), 0, s, *d);
  if (d->dimg) {
    if (warp_win_env == 3) {
      if (c3)
        DVIE_LAUNCH((warp_bwd_pull_kernel<3, 3>), dim3(grid), dim3(256), 0, s, *d);
      else
        DVIE_LAUNCH((warp_bwd_pull_kernel<3, 0>), dim3(grid), dim3(256), 0, s, *d);
    } else {
      if (c3)
        DVIE_LAUNCH((warp_bwd_pull_kernel<4, 3>), dim3(grid), dim3(256), 0, s, *d);
      else
        DVIE_LAUNCH((warp_bwd_pull_kernel<4, 0>), dim3(grid), dim3(256), 0, s, *d);
    }
    const long long quads = ((long long)d->n * d->h * d->w + 3) / 4;
    DVIE_LAUNCH(warp_bwd_far_kernel, dim3((unsigned)std::min<long long>((quads + 255) / 256, 4096)), dim3(256), 0, s, *d);
  }
  DVIE_RETURN_LAUNCH();
}

int dvie_adamax(float* p, const float* g, float* m, float* u, long long n, float clr, float b1, float b2, float eps,
                float wd, void* stream) {
  DVIE_CHECK_ARG(p && g && m && u && n >= 0, "adamax: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(adamax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, u, n, clr, b1, b2,
                     eps, wd, (const float*)nullptr, 0.0, 0.0);
  DVIE_RETURN_LAUNCH();
}

int dvie_adamax_dev(float* p, const float* g, float* m, float* u, long long n, double lr, double b1, double b2,
                    double eps, double wd, const float* step, void* stream) {
  DVIE_CHECK_ARG(p && g && m && u && step && n >= 0, "adamax_dev: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(adamax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, u, n, 0.f,
                     (float)b1, (float)b2, (float)eps, (float)wd, step, lr, b1);
  DVIE_RETURN_LAUNCH();
}

int dvie_step_inc(float* step, void* stream) {
  DVIE_CHECK_ARG(step, "step_inc: null");
  DVIE_LAUNCH(step_inc_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step);
  DVIE_RETURN_LAUNCH();
}

int dvie_scale(float* p, long long n, float s, void* stream) {
  DVIE_CHECK_ARG(p && n >= 0, "scale: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, n, s);
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"

// Lanes of the op-list executor (dvie_op.lane, include/dvie.h): lane 0 is the caller's
// stream; lane 1 (the weight lane) is a side stream of the current device and host thread,
// created on first use at the default (lowest) priority, as the caller's stream.  Events
// are re-recorded at every use: a stream wait binds to the record that precedes it.
namespace {
struct DevLanes {
  hipStream_t side = nullptr;
  hipEvent_t join = nullptr, tail = nullptr;
  bool ok = false;
};
// per host thread (the forward and the autograd backward thread each get their own side
// stream and events, so calls from two threads never re-record each other's events)
thread_local DevLanes dev_lanes[64];

DevLanes* lanes_of_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  DevLanes& d = dev_lanes[dev];
  if (!d.ok) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
    if (hipStreamCreateWithPriority(&d.side, hipStreamNonBlocking, least) != hipSuccess ||
        hipEventCreateWithFlags(&d.join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d.tail, hipEventDisableTiming) != hipSuccess)
      return nullptr;
    d.ok = true;
  }
  return &d;
}

bool lanes_on() {
  const char* e = getenv("DVIE_OP_LANES");
  return !(e && *e == '0');
}

// per-call lane bookkeeping: every data op runs on the caller's stream, so a weight-lane op
// that follows any data op waits for the caller's stream at its current position
struct LaneRun {
  DevLanes* d = nullptr;
  hipStream_t main = nullptr;
  bool tail_fresh = false;  // the weight lane already waits for the caller's current position
  bool used = false;

  hipError_t enter_weight() {
    hipError_t e = hipSuccess;
    if (!tail_fresh) {
      e = hipEventRecord(d->tail, main);
      if (e == hipSuccess) e = hipStreamWaitEvent(d->side, d->tail, 0);
      tail_fresh = true;
    }
    used = true;
    return e;
  }
  hipError_t finish() {
    if (!used) return hipSuccess;
    hipError_t e = hipEventRecord(d->join, d->side);
    return e == hipSuccess ? hipStreamWaitEvent(main, d->join, 0) : e;
  }
};
}  // namespace

extern "C" {

int dvie_run_ops(const dvie_op* ops, int n, void* stream) {
  LaneRun lr;
  lr.main = (hipStream_t)stream;
  // Under stream capture every op stays on the caller's stream: the weight lane's per-run
  // waits become graph edges, and the replayed graph ran 23-33% slower than the one-stream
  // capture (C2 43.7 vs 35.4 ms, C5 224 vs 169 ms per step, profiles/r04v/); eagerly the lane
  // still gains (C2 34.9 vs 35.4 ms).
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(lr.main, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
  const bool lanes = lanes_on() && !capturing;
  auto finish = [&](int rc) {
    if (lr.d) {
      const hipError_t e = lr.finish();
      if (rc == DVIE_OK && e != hipSuccess) {
        set_error("run_ops: lane join failed");
        return (int)e;
      }
    }
    return rc;
  };
  for (int i = 0; i < n; ++i) {
    int rc = DVIE_OK;
    const dvie_op& o = ops[i];
    if (o.lane < 0 || o.lane > 1) {
      set_error("run_ops: lane %d of op %d out of range", o.lane, i);
      return finish(DVIE_EINVAL);
    }
    hipStream_t st = lr.main;
    if (lanes && o.lane == 1) {
      if (!lr.d) lr.d = lanes_of_device();
      if (!lr.d) {
        set_error("run_ops: side stream unavailable");
        return finish(DVIE_EINVAL);
      }
      if (lr.enter_weight() != hipSuccess) {
        set_error("run_ops: weight-lane wait failed at op %d", i);
        return finish(DVIE_EINVAL);
      }
      st = lr.d->side;
    } else {
      lr.tail_fresh = false;  // the caller's stream moves on past the weight lane's wait
    }
    void* s = (void*)st;
#ifdef DVIE_TIMING_DBG
    // timing-only ablation (-DDVIE_TIMING_DBG builds, wrong results): DVIE_SKIP_KINDS = bit mask
    // of op kinds left out, e.g. the weight-gradient reductions, to price them in the step
    static const long long skip_kinds = getenv("DVIE_SKIP_KINDS") ? atoll(getenv("DVIE_SKIP_KINDS")) : 0;
    if ((skip_kinds >> o.kind) & 1) continue;
#endif
    switch (o.kind) {
      case DVIE_OP_CONV: rc = dvie_conv2d_fwd(&o.u.conv, s); break;
      case DVIE_OP_WGRAD: rc = dvie_conv2d_wgrad(&o.u.wgrad, s); break;
      case DVIE_OP_WREDUCE: rc = dvie_wgrad_reduce(&o.u.wreduce, s); break;
      case DVIE_OP_WREDUCE_MULTI: rc = dvie_wgrad_reduce_multi(o.u.wreduce_multi.descs, o.u.wreduce_multi.n, s); break;
      case DVIE_OP_COLSUM: rc = dvie_colsum(&o.u.colsum, s); break;
      case DVIE_OP_EW: rc = dvie_ew(&o.u.ew, s); break;
      case DVIE_OP_LOSS: rc = dvie_loss(&o.u.loss, s); break;
      case DVIE_OP_PACK: rc = dvie_pack_weights(o.u.pack.descs_dev, o.u.pack.n, o.u.pack.blocks, s); break;
      case DVIE_OP_BN_FWD: rc = dvie_bn_fwd(&o.u.bn, s); break;
      case DVIE_OP_BN_BWD: rc = dvie_bn_bwd(&o.u.bn, s); break;
      case DVIE_OP_HEAD_FWD: rc = dvie_head_fwd(&o.u.head, s); break;
      case DVIE_OP_HEAD_BWD: rc = dvie_head_bwd(&o.u.head, s); break;
      case DVIE_OP_ATTN: rc = dvie_attn(&o.u.attn, s); break;
      case DVIE_OP_HEAD3_BWD: rc = dvie_head3_bwd(&o.u.head3, s); break;
      case DVIE_OP_SEGENC_FWD: rc = dvie_segenc_fwd(&o.u.segenc, s); break;
      case DVIE_OP_SEGENC_BWD: rc = dvie_segenc_bwd(&o.u.segenc_bwd, s); break;
      default: set_error("run_ops: unknown op kind %d at %d", o.kind, i); return finish(DVIE_EINVAL);
    }
    if (rc != DVIE_OK) {
      if (rc == DVIE_EINVAL) {
        // keep the message, prefix the op index
        char buf[512];
        snprintf(buf, sizeof(buf), "op %d (kind %d): %s", i, o.kind, dvie_last_error());
        set_error("%s", buf);
      }
      return finish(rc);
    }
  }
  return finish(DVIE_OK);
}

size_t dvie_abi_sizeof(int which) {
  switch (which) {
    case 0: return sizeof(dvie_op);
    case DVIE_OP_CONV: return sizeof(dvie_conv_desc);
    case DVIE_OP_WGRAD: return sizeof(dvie_wgrad_desc);
    case DVIE_OP_WREDUCE: return sizeof(dvie_wreduce_desc);
    case DVIE_OP_WREDUCE_MULTI: return sizeof(dvie_wreduce_multi_desc);
    case DVIE_OP_COLSUM: return sizeof(dvie_colsum_desc);
    case DVIE_OP_EW: return sizeof(dvie_ew_desc);
    case DVIE_OP_LOSS: return sizeof(dvie_loss_desc);
    case DVIE_OP_PACK: return sizeof(dvie_pack_desc);
    case DVIE_OP_BN_FWD: return sizeof(dvie_bn_desc);
    case DVIE_OP_HEAD_FWD: return sizeof(dvie_head_desc);
    case DVIE_OP_ATTN: return sizeof(dvie_attn_desc);
    case DVIE_OP_HEAD3_BWD: return sizeof(dvie_head3_bwd_desc);
    case DVIE_OP_SEGENC_FWD: return sizeof(dvie_segenc_desc);
    case DVIE_OP_SEGENC_BWD: return sizeof(dvie_segenc_bwd_desc);
    case 100: return sizeof(dvie_warp_desc);
    case 101: return sizeof(dvie_softmax_desc);
    case 102: return sizeof(dvie_sn_layer);
    case 103: return sizeof(dvie_clip_desc);
    default: return 0;
  }
}

const char* dvie_version(void) { return "dvie 0.1.0 gfx950"; }

}  // extern "C"
