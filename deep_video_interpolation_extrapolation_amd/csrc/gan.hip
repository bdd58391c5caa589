// gan.hip — the GAN-side kernels of InterGANNet (reference nets/InterGANNet.py:28-117):
//   * BatchNorm2d with training-mode batch statistics (nets/FrameDisc.py:45, VidDisc.py:45,49,
//     HRNet.py:726-789) fused with the following LeakyReLU, forward and backward;
//   * the discriminator head AvgPool2d(p) + view(-1, C).mean(1) (FrameDisc.py:66,74,
//     VidDisc.py:77,83), which averages groups of C consecutive elements of the NCHW-flat
//     pooled tensor (per-sample channel mean only when the pooled map is 1x1);
//   * channel softmax of the segmentation logits (InterGANNet.py:40) and its adjoint;
//   * fused Adam (InterGANTrainer.py:110-112), torch 1.0.1 update form.
// All per-channel reductions use deterministic per-block partials (fp64) and a fold kernel:
// no atomics, identical results run to run.
#include "common.h"

namespace dvie {

constexpr int BN_THREADS = 256;

// mode 0: s1 += x, s2 += x^2                  (forward statistics)
// mode 1: s1 += g, s2 += g * (x - mean[c])     (backward statistics; a = g, b = x)
template <typename TA, typename TB>
__global__ void __launch_bounds__(BN_THREADS) bn_stats_kernel(const TA* __restrict__ a, long long a_ld,
                                                              const TB* __restrict__ b, long long b_ld,
                                                              const float* __restrict__ mean, long long rows, int c,
                                                              long long rows_per_split, double* __restrict__ part,
                                                              int mode) {
  __shared__ double red[BN_THREADS][8];
  const int cg = c >> 2;
  const int lanes = BN_THREADS / cg;
  const int tid = threadIdx.x;
  const int g = tid % cg, rl = tid / cg;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  const long long r0 = (long long)blockIdx.x * rows_per_split;
  const long long r1 = min(rows, r0 + rows_per_split);
  if (rl < lanes) {
    f32x4 mu = {0.f, 0.f, 0.f, 0.f};
    if (mode == 1) mu = *(const f32x4*)(mean + 4 * g);
    for (long long r = r0 + rl; r < r1; r += lanes) {
      const f32x4 va = V4<TA>::load(a + r * a_ld + 4 * g);
      if (mode == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s1[k] += (double)va[k];
          s2[k] += (double)va[k] * (double)va[k];
        }
      } else {
        const f32x4 vb = V4<TB>::load(b + r * b_ld + 4 * g);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s1[k] += (double)va[k];
          s2[k] += (double)va[k] * ((double)vb[k] - (double)mu[k]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[tid][k] = s1[k];
    red[tid][4 + k] = s2[k];
  }
  __syncthreads();
  if (tid < cg) {
    double t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = 0.0;
    for (int l = 0; l < lanes; ++l)
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] += red[l * cg + tid][k];
    double* p = part + (long long)blockIdx.x * 2 * c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[4 * tid + k] = t[k];
      p[c + 4 * tid + k] = t[4 + k];
    }
  }
}

// stats layout (fp32, [8][c]): 0 mean, 1 invstd, 2 scale, 3 shift
__global__ void bn_fold_fwd_kernel(dvie_bn_desc d) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= d.c) return;
  const int c = d.c;
  double mean, var;
  if (d.training) {
    double s1 = 0.0, s2 = 0.0;
    for (int s = 0; s < d.splits; ++s) {
      s1 += d.partial[(long long)s * 2 * c + ch];
      s2 += d.partial[(long long)s * 2 * c + c + ch];
    }
    const double M = (double)d.rows;
    mean = s1 / M;
    var = s2 / M - mean * mean;
    if (var < 0.0) var = 0.0;
    if (d.running_mean) {
      const double m = d.momentum;
      d.running_mean[ch] = (float)((1.0 - m) * d.running_mean[ch] + m * mean);
      const double unb = d.rows > 1 ? var * M / (M - 1.0) : var;
      d.running_var[ch] = (float)((1.0 - m) * d.running_var[ch] + m * unb);
    }
  } else {
    mean = d.running_mean[ch];
    var = d.running_var[ch];
  }
  const float inv = (float)(1.0 / sqrt(var + (double)d.eps));
  const float gam = d.gamma ? d.gamma[ch] : 1.f;
  const float bet = d.beta ? d.beta[ch] : 0.f;
  const float scale = gam * inv;
  d.stats[ch] = (float)mean;
  d.stats[c + ch] = inv;
  d.stats[2 * c + ch] = scale;
  d.stats[3 * c + ch] = bet - (float)mean * scale;
}

__global__ void bn_fold_bwd_kernel(dvie_bn_desc d) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= d.c) return;
  const int c = d.c;
  double sg = 0.0, sgc = 0.0;
  for (int s = 0; s < d.splits; ++s) {
    sg += d.partial[(long long)s * 2 * c + ch];
    sgc += d.partial[(long long)s * 2 * c + c + ch];
  }
  const double M = (double)d.rows;
  const double inv = d.stats[c + ch];
  const double mean = d.stats[ch];
  const double gam = d.gamma ? d.gamma[ch] : 1.0;
  if (d.dgamma) d.dgamma[ch] = (float)(sgc * inv + (d.accumulate ? (double)d.dgamma[ch] : 0.0));
  if (d.dbeta) d.dbeta[ch] = (float)(sg + (d.accumulate ? (double)d.dbeta[ch] : 0.0));
  // dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)) = A*(g - mg) + B*(x - mean).
  // The true dx is typically orders of magnitude below g (BatchNorm removes the mean and
  // the xhat-correlated part), so the apply kernel evaluates it in fp64 from fp64
  // coefficients, written over this channel's own (already consumed) partial slots.
  const double A = gam * inv;
  const double B = -A * inv * inv * sgc / M;
  d.partial[ch] = A;
  d.partial[c + ch] = B;
  d.partial[2 * c + ch] = sg / M;
  d.partial[3 * c + ch] = mean;
}

// forward: y = act(x*scale + shift); backward (bwd=1): dx (+)= A*(g - mg) + B*(x - mean)
template <typename TX, typename T>
__global__ void bn_apply_kernel(dvie_bn_desc d, int bwd) {
  const int cg = d.c >> 2;
  const long long total = d.rows * cg;
  const int c = d.c;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cg;
    const int ch = (int)(i - r * cg) * 4;
    const f32x4 xv = V4<TX>::load((const TX*)d.x + r * d.x_ld + ch);
    f32x4 o;
    if (!bwd) {
      const f32x4 sc = *(const f32x4*)(d.stats + 2 * c + ch);
      const f32x4 sh = *(const f32x4*)(d.stats + 3 * c + ch);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = act_fwd(xv[k] * sc[k] + sh[k], d.act, d.alpha);
      V4<T>::store((T*)d.y + r * d.y_ld + ch, o);
    } else {
      const f32x4 gv = V4<T>::load((const T*)d.g + r * d.g_ld + ch);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double A = d.partial[ch + k], B = d.partial[c + ch + k];
        const double mg = d.partial[2 * c + ch + k], mu = d.partial[3 * c + ch + k];
        o[k] = (float)(A * ((double)gv[k] - mg) + B * ((double)xv[k] - mu));
      }
      T* dp = (T*)d.dx + r * d.dx_ld + ch;
      if (d.beta_dx) {
        const f32x4 old = V4<T>::load(dp);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] += old[k];
      }
      V4<T>::store(dp, o);
    }
  }
}

// ---- discriminator head ----
template <typename T>
__global__ void head_pool_kernel(dvie_head_desc d) {
  const int p = d.pool, hp = d.h / p, wp = d.w / p, c = d.c;
  const long long total = (long long)d.n * hp * wp * c;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    // NHWC decode (channel fastest: coalesced reads), NCHW-flat write
    const int ch = (int)(i % c);
    long long r = i / c;
    const int px = (int)(r % wp);
    r /= wp;
    const int py = (int)(r % hp);
    const int b = (int)(r / hp);
    float s = 0.f;
    for (int yy = 0; yy < p; ++yy)
      for (int xx = 0; xx < p; ++xx) {
        const long long pix = ((long long)b * d.h + py * p + yy) * d.w + px * p + xx;
        const T* q = (const T*)d.x + pix * d.x_ld + ch;
        if constexpr (sizeof(T) == 4)
          s += *(const float*)q;
        else
          s += bf2f(*(const bf16_t*)q);
      }
    d.pooled[(((long long)b * c + ch) * hp + py) * wp + px] = s / (float)(p * p);
  }
}

__global__ void head_mean_kernel(dvie_head_desc d) {
  const int hp = d.h / d.pool, wp = d.w / d.pool;
  const long long rows = (long long)d.n * hp * wp;  // = n*c*hp*wp / c
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < rows;
       r += (long long)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < d.c; ++k) s += d.pooled[r * d.c + k];
    d.out[r] = (float)(s / d.c);
  }
}

template <typename T>
__global__ void head_bwd_kernel(dvie_head_desc d) {
  const int p = d.pool, hp = d.h / p, wp = d.w / p, c = d.c;
  const int cg = c >> 2;
  const long long total = (long long)d.n * d.h * d.w * cg;
  const float inv = 1.f / ((float)c * p * p);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cg) * 4;
    long long r = i / cg;
    const int x = (int)(r % d.w);
    r /= d.w;
    const int y = (int)(r % d.h);
    const int b = (int)(r / d.h);
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (y < hp * p && x < wp * p) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long long e = (((long long)b * c + ch + k) * hp + y / p) * wp + x / p;
        o[k] = d.gout[e / c] * inv;
      }
    }
    T* q = (T*)d.gx + (((long long)b * d.h + y) * d.w + x) * d.gx_ld + ch;
    if (d.beta) {
      const f32x4 old = V4<T>::load(q);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] += old[k];
    }
    V4<T>::store(q, o);
  }
}

// ---- channel softmax (fp32, arbitrary NCHW strides in, contiguous NCHW out) ----
__global__ void softmax_fwd_kernel(dvie_softmax_desc d) {
  const long long hw = (long long)d.h * d.w;
  const long long total = (long long)d.n * hw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / hw, pix = i - b * hw;
    const int y = (int)(pix / d.w), x = (int)(pix - (long long)y * d.w);
    const float* src = d.x + b * d.sn + y * d.sh + x * d.sw;
    float m = -INFINITY;
    for (int k = 0; k < d.c; ++k) m = fmaxf(m, src[k * d.sc]);
    float s = 0.f;
    for (int k = 0; k < d.c; ++k) s += expf(src[k * d.sc] - m);
    const float inv = 1.f / s;
    float* dst = d.y + b * d.c * hw + pix;
    for (int k = 0; k < d.c; ++k) dst[k * hw] = expf(src[k * d.sc] - m) * inv;
  }
}

__global__ void softmax_bwd_kernel(dvie_softmax_desc d) {
  const long long hw = (long long)d.h * d.w;
  const long long total = (long long)d.n * hw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / hw, pix = i - b * hw;
    const long long base = b * d.c * hw + pix;
    float dot = 0.f;
    for (int k = 0; k < d.c; ++k) dot += d.gy[base + k * hw] * d.y[base + k * hw];
    for (int k = 0; k < d.c; ++k) {
      const long long o = base + k * hw;
      const float v = d.y[o] * (d.gy[o] - dot);
      d.gx[o] = d.beta ? d.gx[o] + v : v;
    }
  }
}

// torch 1.0.1 Adam: m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g;
// p -= step_size * m / (sqrt(v) + eps), step_size = lr*sqrt(1-b2^t)/(1-b1^t) (host).
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float step_size, float b1, float b2, float eps,
                            float wd, const float* __restrict__ stepp, double lr, double b1d, double b2d) {
  if (stepp) {  // device-resident step count (graph-captured steps), host-identical doubles
    const double t = (double)stepp[0];
    step_size = (float)(lr * sqrt(1.0 - pow(b2d, t)) / (1.0 - pow(b1d, t)));
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float pv = p[i];
    float gr = g[i];
    if (wd != 0.f) gr += wd * pv;
    const float mn = m[i] * b1 + (1.f - b1) * gr;
    const float vn = v[i] * b2 + (1.f - b2) * gr * gr;
    m[i] = mn;
    v[i] = vn;
    p[i] = pv - step_size * (mn / (sqrtf(vn) + eps));
  }
}

static int grid_1d(long long n, int per = 256) {
  long long b = (n + per - 1) / per;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

static int bn_check(const dvie_bn_desc* d) {
  DVIE_CHECK_ARG(d && d->x && d->stats && d->rows > 0 && d->c > 0 && d->c % 4 == 0 && d->c <= 4 * BN_THREADS,
                 "bn: bad args (c %d must be a multiple of 4, <= %d)", d ? d->c : -1, 4 * BN_THREADS);
  DVIE_CHECK_ARG(d->x_ld % 4 == 0 && d->x_ld >= d->c, "bn: x_ld");
  DVIE_CHECK_ARG(d->dtype == DVIE_F32 || d->dtype == DVIE_BF16, "bn: dtype");
  return DVIE_OK;
}

// x (the BatchNorm input, a conv output) may be fp32 while y / g / dx have the compute
// dtype: bf16 storage of a pre-normalisation tensor whose |mean| >> std would cost
// 2^-9 * |mean| / std relative precision in x - mean.
template <typename TX, typename T>
static void bn_launch(const dvie_bn_desc* d, hipStream_t st, int bwd) {
  const long long rps = (d->rows + d->splits - 1) / d->splits;
  if (!bwd) {
    if (d->training)
      DVIE_LAUNCH((bn_stats_kernel<TX, TX>), dim3(d->splits), dim3(BN_THREADS), 0, st, (const TX*)d->x,
                         d->x_ld, (const TX*)nullptr, 0LL, (const float*)nullptr, d->rows, d->c, rps, d->partial, 0);
    DVIE_LAUNCH(bn_fold_fwd_kernel, dim3((d->c + 63) / 64), dim3(64), 0, st, *d);
  } else {
    DVIE_LAUNCH((bn_stats_kernel<T, TX>), dim3(d->splits), dim3(BN_THREADS), 0, st, (const T*)d->g, d->g_ld,
                       (const TX*)d->x, d->x_ld, (const float*)d->stats, d->rows, d->c, rps, d->partial, 1);
    DVIE_LAUNCH(bn_fold_bwd_kernel, dim3((d->c + 63) / 64), dim3(64), 0, st, *d);
  }
  const long long n4 = d->rows * (d->c / 4);
  DVIE_LAUNCH((bn_apply_kernel<TX, T>), dim3(grid_1d(n4)), dim3(256), 0, st, *d, bwd);
}

static void bn_dispatch(const dvie_bn_desc* d, hipStream_t st, int bwd) {
  if (d->dtype == DVIE_BF16) {
    if (d->x_f32)
      bn_launch<float, bf16_t>(d, st, bwd);
    else
      bn_launch<bf16_t, bf16_t>(d, st, bwd);
  } else {
    bn_launch<float, float>(d, st, bwd);
  }
}

}  // namespace dvie

using namespace dvie;

extern "C" {

int dvie_bn_partial_splits(const dvie_bn_desc* d) {
  if (!d || d->rows <= 0) return 1;
  long long s = d->rows / 2048;
  if (s < 1) s = 1;
  if (s > 512) s = 512;
  return (int)s;
}

int dvie_bn_fwd(const dvie_bn_desc* d, void* stream) {
  int rc = bn_check(d);
  if (rc) return rc;
  DVIE_CHECK_ARG(d->y && d->y_ld % 4 == 0, "bn fwd: y");
  if (d->training)
    DVIE_CHECK_ARG(d->partial && d->splits >= 1, "bn fwd: partial workspace");
  else
    DVIE_CHECK_ARG(d->running_mean && d->running_var, "bn eval: running statistics");
  bn_dispatch(d, (hipStream_t)stream, 0);
  DVIE_RETURN_LAUNCH();
}

int dvie_bn_bwd(const dvie_bn_desc* d, void* stream) {
  int rc = bn_check(d);
  if (rc) return rc;
  DVIE_CHECK_ARG(d->training, "bn bwd: only training-mode statistics have a backward here");
  DVIE_CHECK_ARG(d->g && d->dx && d->partial && d->splits >= 1 && d->g_ld % 4 == 0 && d->dx_ld % 4 == 0,
                 "bn bwd: args");
  bn_dispatch(d, (hipStream_t)stream, 1);
  DVIE_RETURN_LAUNCH();
}

int dvie_head_fwd(const dvie_head_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->x && d->out && d->pooled && d->pool > 0 && d->h >= d->pool && d->w >= d->pool && d->c > 0,
                 "head fwd: args (h %d w %d pool %d)", d ? d->h : -1, d ? d->w : -1, d ? d->pool : -1);
  hipStream_t st = (hipStream_t)stream;
  const long long np = (long long)d->n * (d->h / d->pool) * (d->w / d->pool);
  if (d->dtype == DVIE_BF16)
    DVIE_LAUNCH(head_pool_kernel<bf16_t>, dim3(grid_1d(np * d->c)), dim3(256), 0, st, *d);
  else
    DVIE_LAUNCH(head_pool_kernel<float>, dim3(grid_1d(np * d->c)), dim3(256), 0, st, *d);
  DVIE_LAUNCH(head_mean_kernel, dim3(grid_1d(np)), dim3(256), 0, st, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_head_bwd(const dvie_head_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->gx && d->gout && d->pool > 0 && d->c % 4 == 0 && d->gx_ld % 4 == 0, "head bwd: args");
  hipStream_t st = (hipStream_t)stream;
  const long long n4 = (long long)d->n * d->h * d->w * (d->c / 4);
  if (d->dtype == DVIE_BF16)
    DVIE_LAUNCH(head_bwd_kernel<bf16_t>, dim3(grid_1d(n4)), dim3(256), 0, st, *d);
  else
    DVIE_LAUNCH(head_bwd_kernel<float>, dim3(grid_1d(n4)), dim3(256), 0, st, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_softmax_fwd(const dvie_softmax_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->x && d->y && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "softmax fwd: args");
  DVIE_LAUNCH(softmax_fwd_kernel, dim3(grid_1d((long long)d->n * d->h * d->w)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_softmax_bwd(const dvie_softmax_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->y && d->gy && d->gx && d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0, "softmax bwd: args");
  DVIE_LAUNCH(softmax_bwd_kernel, dim3(grid_1d((long long)d->n * d->h * d->w)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

int dvie_adam(float* p, const float* g, float* m, float* v, long long n, float step_size, float b1, float b2,
              float eps, float wd, void* stream) {
  DVIE_CHECK_ARG(p && g && m && v && n >= 0, "adam: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(adam_kernel, dim3(grid_1d(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, step_size, b1,
                     b2, eps, wd, (const float*)nullptr, 0.0, 0.0, 0.0);
  DVIE_RETURN_LAUNCH();
}

int dvie_adam_dev(float* p, const float* g, float* m, float* v, long long n, double lr, double b1, double b2,
                  double eps, double wd, const float* step, void* stream) {
  DVIE_CHECK_ARG(p && g && m && v && step && n >= 0, "adam_dev: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(adam_kernel, dim3(grid_1d(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, 0.f,
                     (float)b1, (float)b2, (float)eps, (float)wd, step, lr, b1, b2);
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"
