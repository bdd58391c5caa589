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

__global__ void warp_fwd_kernel(const dvie_warp_desc p) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * hw;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / hw);
    const float gx = linspace_pm1(x, p.w) - p.flow[((long long)n * 2 + 0) * hw + (long long)y * p.w + x];
    const float gy = linspace_pm1(y, p.h) - p.flow[((long long)n * 2 + 1) * hw + (long long)y * p.w + x];
    const float ix = unnorm(gx, p.w, p.align_corners), iy = unnorm(gy, p.h, p.align_corners);
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    const int x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((float)x1 - ix) * ((float)y1 - iy), wne = (ix - (float)x0) * ((float)y1 - iy);
    const float wsw = ((float)x1 - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
    const bool vx0 = x0 >= 0 && x0 < p.w, vx1 = x1 >= 0 && x1 < p.w;
    const bool vy0 = y0 >= 0 && y0 < p.h, vy1 = y1 >= 0 && y1 < p.h;
    for (int c = 0; c < p.c; ++c) {
      const float* im = p.img + ((long long)n * p.c + c) * hw;
      float v = 0.f;
      if (vy0 && vx0) v += im[(long long)y0 * p.w + x0] * wnw;
      if (vy0 && vx1) v += im[(long long)y0 * p.w + x1] * wne;
      if (vy1 && vx0) v += im[(long long)y1 * p.w + x0] * wsw;
      if (vy1 && vx1) v += im[(long long)y1 * p.w + x1] * wse;
      p.out[((long long)n * p.c + c) * hw + (long long)y * p.w + x] = v;
    }
  }
}

__global__ void warp_bwd_kernel(const dvie_warp_desc p) {
  const long long hw = (long long)p.h * p.w;
  const long long total = (long long)p.n * hw;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / hw);
    const long long fo = (long long)y * p.w + x;
    const float gx = linspace_pm1(x, p.w) - p.flow[((long long)n * 2 + 0) * hw + fo];
    const float gy = linspace_pm1(y, p.h) - p.flow[((long long)n * 2 + 1) * hw + fo];
    const float ix = unnorm(gx, p.w, p.align_corners), iy = unnorm(gy, p.h, p.align_corners);
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    const int x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((float)x1 - ix) * ((float)y1 - iy), wne = (ix - (float)x0) * ((float)y1 - iy);
    const float wsw = ((float)x1 - ix) * (iy - (float)y0), wse = (ix - (float)x0) * (iy - (float)y0);
    const bool vx0 = x0 >= 0 && x0 < p.w, vx1 = x1 >= 0 && x1 < p.w;
    const bool vy0 = y0 >= 0 && y0 < p.h, vy1 = y1 >= 0 && y1 < p.h;
    float gix = 0.f, giy = 0.f;
    for (int c = 0; c < p.c; ++c) {
      const long long base = ((long long)n * p.c + c) * hw;
      const float go = p.dout[base + fo];
      const float* im = p.img + base;
      if (vy0 && vx0) {
        const float v = im[(long long)y0 * p.w + x0];
        gix -= v * ((float)y1 - iy) * go;
        giy -= v * ((float)x1 - ix) * go;
        if (p.dimg) atomicAdd(p.dimg + base + (long long)y0 * p.w + x0, wnw * go);
      }
      if (vy0 && vx1) {
        const float v = im[(long long)y0 * p.w + x1];
        gix += v * ((float)y1 - iy) * go;
        giy -= v * (ix - (float)x0) * go;
        if (p.dimg) atomicAdd(p.dimg + base + (long long)y0 * p.w + x1, wne * go);
      }
      if (vy1 && vx0) {
        const float v = im[(long long)y1 * p.w + x0];
        gix -= v * (iy - (float)y0) * go;
        giy += v * ((float)x1 - ix) * go;
        if (p.dimg) atomicAdd(p.dimg + base + (long long)y1 * p.w + x0, wsw * go);
      }
      if (vy1 && vx1) {
        const float v = im[(long long)y1 * p.w + x1];
        gix += v * (iy - (float)y0) * go;
        giy += v * (ix - (float)x0) * go;
        if (p.dimg) atomicAdd(p.dimg + base + (long long)y1 * p.w + x1, wse * go);
      }
    }
    if (p.dflow) {
      const float sx = p.align_corners ? (float)(p.w - 1) / 2.f : (float)p.w / 2.f;
      const float sy = p.align_corners ? (float)(p.h - 1) / 2.f : (float)p.h / 2.f;
      p.dflow[((long long)n * 2 + 0) * hw + fo] = -gix * sx;
      p.dflow[((long long)n * 2 + 1) * hw + fo] = -giy * sy;
    }
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
  hipLaunchKernelGGL(warp_fwd_kernel, dim3(grid_for((long long)d->n * d->h * d->w)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_warp_bwd(const dvie_warp_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->flow && d->dout && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "warp: args");
  hipLaunchKernelGGL(warp_bwd_kernel, dim3(grid_for((long long)d->n * d->h * d->w)), dim3(256), 0,
                     (hipStream_t)stream, *d);
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
