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

__device__ __forceinline__ float warp_sample(const float* __restrict__ im, const WarpTap& t, int w) {
  float v = 0.f;
  if (t.vy0 && t.vx0) v += im[(long long)t.y0 * w + t.x0] * t.wnw;
  if (t.vy0 && t.vx1) v += im[(long long)t.y0 * w + t.x0 + 1] * t.wne;
  if (t.vy1 && t.vx0) v += im[(long long)(t.y0 + 1) * w + t.x0] * t.wsw;
  if (t.vy1 && t.vx1) v += im[(long long)(t.y0 + 1) * w + t.x0 + 1] * t.wse;
  return v;
}

__global__ void warp_fwd_kernel(const dvie_warp_desc p) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * hw;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / hw);
    const long long fo = (long long)y * p.w + x;
    const WarpTap t = warp_tap(x, y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo], p.w,
                               p.h, p.align_corners);
    for (int c = 0; c < p.c; ++c) {
      const long long base = ((long long)n * p.c + c) * hw;
      p.out[base + fo] = warp_sample(p.img + base, t, p.w);
    }
  }
}

// 4 consecutive pixels per thread (w % 4 == 0): 16-byte flow loads and output stores, 4x
// the independent gathers in flight per thread; per-pixel arithmetic identical to the above
__global__ __launch_bounds__(256) void warp_fwd4_kernel(const dvie_warp_desc p) {
  const int wq = p.w >> 2;
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * p.h * wq;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int xq = (int)(e % wq);
    const long long r = e / wq;
    const int y = (int)(r % p.h), n = (int)(r / p.h);
    const int x = 4 * xq;
    const long long fo = (long long)y * p.w + x;
    const f32x4 fx = *(const f32x4*)(p.flow + (long long)n * 2 * hw + fo);
    const f32x4 fy = *(const f32x4*)(p.flow + ((long long)n * 2 + 1) * hw + fo);
    WarpTap t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = warp_tap(x + k, y, fx[k], fy[k], p.w, p.h, p.align_corners);
    for (int c = 0; c < p.c; ++c) {
      const long long base = ((long long)n * p.c + c) * hw;
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = warp_sample(p.img + base, t[k], p.w);
      *(f32x4*)(p.out + base + fo) = o;
    }
  }
}

// ---- backward ----
// d/d(img) of one bilinear corner, and the flow-gradient terms, per channel (order of the
// reference autograd: corners nw, ne, sw, se)
template <typename Scatter>
__device__ __forceinline__ void warp_bwd_pixel(const float* __restrict__ im, float go, const WarpTap& t, int w,
                                               float& gix, float& giy, Scatter&& scatter) {
  const int x1 = t.x0 + 1, y1 = t.y0 + 1;
  if (t.vy0 && t.vx0) {
    const float v = im[(long long)t.y0 * w + t.x0];
    gix -= v * ((float)y1 - t.iy) * go;
    giy -= v * ((float)x1 - t.ix) * go;
    scatter(t.y0, t.x0, t.wnw * go);
  }
  if (t.vy0 && t.vx1) {
    const float v = im[(long long)t.y0 * w + x1];
    gix += v * ((float)y1 - t.iy) * go;
    giy -= v * (t.ix - (float)t.x0) * go;
    scatter(t.y0, x1, t.wne * go);
  }
  if (t.vy1 && t.vx0) {
    const float v = im[(long long)y1 * w + t.x0];
    gix -= v * (t.iy - (float)t.y0) * go;
    giy += v * ((float)x1 - t.ix) * go;
    scatter(y1, t.x0, t.wsw * go);
  }
  if (t.vy1 && t.vx1) {
    const float v = im[(long long)y1 * w + x1];
    gix += v * (t.iy - (float)t.y0) * go;
    giy += v * (t.ix - (float)t.x0) * go;
    scatter(y1, x1, t.wse * go);
  }
}

__device__ __forceinline__ void warp_store_dflow(const dvie_warp_desc& p, int n, long long fo, float gix, float giy) {
  const long long hw = (long long)p.h * p.w;
  const float sx = p.align_corners ? (float)(p.w - 1) / 2.f : (float)p.w / 2.f;
  const float sy = p.align_corners ? (float)(p.h - 1) / 2.f : (float)p.h / 2.f;
  p.dflow[((long long)n * 2 + 0) * hw + fo] = -gix * sx;
  p.dflow[((long long)n * 2 + 1) * hw + fo] = -giy * sy;
}

// one global atomic per corner (no workspace)
__global__ void warp_bwd_kernel(const dvie_warp_desc p) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * hw;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / hw);
    const long long fo = (long long)y * p.w + x;
    const WarpTap t = warp_tap(x, y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo], p.w,
                               p.h, p.align_corners);
    float gix = 0.f, giy = 0.f;
    for (int c = 0; c < p.c; ++c) {
      const long long base = ((long long)n * p.c + c) * hw;
      warp_bwd_pixel(p.img + base, p.dout[base + fo], t, p.w, gix, giy, [&](int yy, int xx, float v) {
        if (p.dimg) atomicAdd(p.dimg + base + (long long)yy * p.w + xx, v);
      });
    }
    if (p.dflow) warp_store_dflow(p, n, fo, gix, giy);
  }
}

// tiled image gradient: a workgroup owns WT_H x WT_W output pixels (4 per thread) and
// accumulates their corner contributions in an LDS copy of its region (the tile grown by
// WT_M pixels on every side), WT_CB channels at a time; the region is then stored to the
// workspace and warp_bwd_gather_kernel sums the (at most 4) regions covering each pixel.
constexpr int WT_W = 64, WT_H = 16, WT_M = 4, WT_CB = 4;
constexpr int WT_RH = WT_H + 2 * WT_M, WT_RW = WT_W + 2 * WT_M, WT_CELLS = WT_RH * WT_RW;

__global__ __launch_bounds__(256) void warp_bwd_tile_kernel(const dvie_warp_desc p, int tiles_x, int tiles_y) {
  __shared__ float acc[WT_CB * WT_CELLS];
  const int tx = blockIdx.x % tiles_x;
  const int ty = (blockIdx.x / tiles_x) % tiles_y;
  const int n = blockIdx.x / (tiles_x * tiles_y);
  const int x = tx * WT_W + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int oy = ty * WT_H - WT_M, ox = tx * WT_W - WT_M;  // region origin
  const long long hw = (long long)p.h * p.w;
  WarpTap t[WT_H / 4];
  bool live[WT_H / 4];
  float gix[WT_H / 4], giy[WT_H / 4];
#pragma unroll
  for (int k = 0; k < WT_H / 4; ++k) {
    const int y = ty * WT_H + rg + 4 * k;
    live[k] = x < p.w && y < p.h;
    gix[k] = giy[k] = 0.f;
    if (live[k]) {
      const long long fo = (long long)y * p.w + x;
      t[k] = warp_tap(x, y, p.flow[(long long)n * 2 * hw + fo], p.flow[((long long)n * 2 + 1) * hw + fo], p.w, p.h,
                      p.align_corners);
    }
  }
  float* region = p.ws + (((long long)n * tiles_y + ty) * tiles_x + tx) * (long long)p.c * WT_CELLS;
  for (int c0 = 0; c0 < p.c; c0 += WT_CB) {
    const int cb = p.c - c0 < WT_CB ? p.c - c0 : WT_CB;
    for (int i = threadIdx.x; i < cb * WT_CELLS; i += 256) acc[i] = 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < WT_H / 4; ++k) {
      if (!live[k]) continue;
      const long long fo = (long long)(ty * WT_H + rg + 4 * k) * p.w + x;
      for (int cc = 0; cc < cb; ++cc) {
        const long long base = ((long long)n * p.c + c0 + cc) * hw;
        float* lds = acc + cc * WT_CELLS;
        warp_bwd_pixel(p.img + base, p.dout[base + fo], t[k], p.w, gix[k], giy[k], [&](int yy, int xx, float v) {
          const int ly = yy - oy, lx = xx - ox;
          if ((unsigned)ly < (unsigned)WT_RH && (unsigned)lx < (unsigned)WT_RW)
            atomicAdd(lds + ly * WT_RW + lx, v);
          else
            atomicAdd(p.dimg + base + (long long)yy * p.w + xx, v);  // far sample: rare
        });
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < cb * WT_CELLS; i += 256) region[(long long)c0 * WT_CELLS + i] = acc[i];
    __syncthreads();
  }
  if (p.dflow) {
#pragma unroll
    for (int k = 0; k < WT_H / 4; ++k)
      if (live[k]) warp_store_dflow(p, n, (long long)(ty * WT_H + rg + 4 * k) * p.w + x, gix[k], giy[k]);
  }
}

__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ __launch_bounds__(256) void warp_bwd_gather_kernel(const dvie_warp_desc p, int tiles_x, int tiles_y) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * p.c * hw;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const long long nc = e / hw;
    const int c = (int)(nc % p.c), n = (int)(nc / p.c);
    int ty0 = floordiv(y - WT_M, WT_H), ty1 = (y + WT_M) / WT_H;
    int tx0 = floordiv(x - WT_M, WT_W), tx1 = (x + WT_M) / WT_W;
    ty0 = ty0 < 0 ? 0 : ty0;
    tx0 = tx0 < 0 ? 0 : tx0;
    ty1 = ty1 > tiles_y - 1 ? tiles_y - 1 : ty1;
    tx1 = tx1 > tiles_x - 1 ? tiles_x - 1 : tx1;
    float s = p.dimg[e];  // far samples (global atomics of the tile pass)
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) {
        const int ly = y - (ty * WT_H - WT_M), lx = x - (tx * WT_W - WT_M);
        s += p.ws[((((long long)n * tiles_y + ty) * tiles_x + tx) * p.c + c) * WT_CELLS + ly * WT_RW + lx];
      }
    p.dimg[e] = s;
  }
}

__global__ void adamax_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                              float* __restrict__ u, long long n, float clr, float b1, float b2, float eps,
                              float wd) {
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
  const bool v4 = d->w % 4 == 0 && (((uintptr_t)d->flow | (uintptr_t)d->out) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(warp_fwd4_kernel, dim3(grid_for((long long)d->n * d->h * (d->w / 4))), dim3(256), 0,
                       (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(warp_fwd_kernel, dim3(grid_for((long long)d->n * d->h * d->w)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

static void warp_tiles(const dvie_warp_desc* d, int& tx, int& ty) {
  tx = (d->w + WT_W - 1) / WT_W;
  ty = (d->h + WT_H - 1) / WT_H;
}

size_t dvie_warp_ws_floats(const dvie_warp_desc* d) {
  if (!d || d->n <= 0 || d->c <= 0 || d->h <= 0 || d->w <= 0) return 0;
  int tx, ty;
  warp_tiles(d, tx, ty);
  return (size_t)d->n * ty * tx * d->c * WT_CELLS;
}

int dvie_warp_bwd(const dvie_warp_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->flow && d->dout && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "warp: args");
  hipStream_t s = (hipStream_t)stream;
  if (d->ws && d->dimg) {
    int tx, ty;
    warp_tiles(d, tx, ty);
    const long long blocks = (long long)d->n * ty * tx;
    DVIE_CHECK_ARG(blocks < (1LL << 31), "warp: grid");
    hipLaunchKernelGGL(warp_bwd_tile_kernel, dim3((unsigned)blocks), dim3(256), 0, s, *d, tx, ty);
    hipLaunchKernelGGL(warp_bwd_gather_kernel, dim3(grid_for((long long)d->n * d->c * d->h * d->w)), dim3(256), 0, s,
                       *d, tx, ty);
  } else {
    hipLaunchKernelGGL(warp_bwd_kernel, dim3(grid_for((long long)d->n * d->h * d->w)), dim3(256), 0, s, *d);
  }
  DVIE_RETURN_LAUNCH();
}

int dvie_adamax(float* p, const float* g, float* m, float* u, long long n, float clr, float b1, float b2, float eps,
                float wd, void* stream) {
  DVIE_CHECK_ARG(p && g && m && u && n >= 0, "adamax: args");
  if (n == 0) return DVIE_OK;
  hipLaunchKernelGGL(adamax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, u, n, clr, b1, b2,
                     eps, wd);
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
    case 100: return sizeof(dvie_warp_desc);
    case 101: return sizeof(dvie_softmax_desc);
    case 102: return sizeof(dvie_sn_layer);
    default: return 0;
  }
}

const char* dvie_version(void) { return "dvie 0.1.0 gfx950"; }

}  // extern "C"
