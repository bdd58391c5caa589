// Loss / metric reductions (fp32 math, double cross-block accumulation, deterministic):
// L1, gradient-difference (GDL), SSIM (11x11 gaussian, separable, LDS-tiled), per-sample
// MSE (PSNR), softmax cross-entropy against argmax(one-hot), the VGG feature L1, and the
// validation metrics VGG feature cosine and IoU (pixel accuracy).
// Each kernel writes per-block partial sums; a one-block kernel folds them into the
// output scalar(s).  When a gradient buffer is given, the kernels also write
// d(weight*loss)/d(pred) in NCHW-contiguous fp32 (the autograd wrappers scale it by
// the incoming gradient).
//
// Reference: losses.py:18-48 (_ssim / create_window), 63-87 (SSIM), 103-116 (PSNR),
// 122-131 (IoU), 137-151 (GDLLoss), 157-180 (VGGLoss feature L1), 182-207 (VGGCosineLoss),
// nn.L1Loss (losses.py:224) and
// nn.CrossEntropyLoss (runners/InterTrainer.py:75,414).
#include "common.h"

namespace dvie {

constexpr int RB = 256;  // reduction block

__device__ __forceinline__ double block_sum(double v, double* sh) {
  const int tid = threadIdx.x;
  // wave reduction
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((tid & 63) == 0) sh[tid >> 6] = v;
  __syncthreads();
  double t = 0.0;
  if (tid == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ float sgnf(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }

struct Shape {
  long long sn, sc, sh, sw;
  __device__ __forceinline__ long long at(int n, int c, int y, int x) const {
    return (long long)n * sn + (long long)c * sc + (long long)y * sh + (long long)x * sw;
  }
};

// elementwise L1 / GDL / MSE over (B, C, H, W) with x fastest
__global__ __launch_bounds__(RB) void l1gdl_kernel(const dvie_loss_desc p, int per_sample_blocks) {
  __shared__ double sh[RB / 64];
  const float* a = (const float*)p.a;
  const float* b = (const float*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const long long per = (long long)p.ch * p.h * p.w;
  long long lo = 0, hi = (long long)p.bsz * per, stride = (long long)gridDim.x * blockDim.x;
  long long start = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (p.kind == DVIE_LOSS_MSE) {  // blocks partitioned per sample
    const int smp = blockIdx.x / per_sample_blocks;
    lo = (long long)smp * per;
    hi = lo + per;
    start = lo + (long long)(blockIdx.x % per_sample_blocks) * blockDim.x + threadIdx.x;
    stride = (long long)per_sample_blocks * blockDim.x;
  }
  const double nx = (double)p.bsz * p.ch * p.h * (p.w - 1), ny = (double)p.bsz * p.ch * (p.h - 1) * p.w;
  const double nall = (double)p.bsz * per;
  double acc = 0.0;
  for (long long e = start; e < hi; e += stride) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int c = (int)((e / ((long long)p.w * p.h)) % p.ch);
    const int n = (int)(e / per);
    const float av = a[sa.at(n, c, y, x)], bv = b[sb.at(n, c, y, x)];
    const float d = av - bv;
    float g = 0.f;
    if (p.kind == DVIE_LOSS_L1) {
      acc += fabsf(d);
      g = sgnf(d) / (float)nall;
    } else if (p.kind == DVIE_LOSS_MSE) {
      acc += (double)(d * d);
    } else {  // GDL
      float gx = 0.f, gy = 0.f;
      if (x + 1 < p.w) {
        const float dx = (a[sa.at(n, c, y, x + 1)] - av) - (b[sb.at(n, c, y, x + 1)] - bv);
        acc += fabs((double)dx) / (2.0 * nx);
        gx -= sgnf(dx);
      }
      if (x > 0) {
        const float dxm = (av - a[sa.at(n, c, y, x - 1)]) - (bv - b[sb.at(n, c, y, x - 1)]);
        gx += sgnf(dxm);
      }
      if (y + 1 < p.h) {
        const float dy = (a[sa.at(n, c, y + 1, x)] - av) - (b[sb.at(n, c, y + 1, x)] - bv);
        acc += fabs((double)dy) / (2.0 * ny);
        gy -= sgnf(dy);
      }
      if (y > 0) {
        const float dym = (av - a[sa.at(n, c, y - 1, x)]) - (bv - b[sb.at(n, c, y - 1, x)]);
        gy += sgnf(dym);
      }
      g = (float)(gx / (2.0 * nx) + gy / (2.0 * ny));
    }
    if (p.grad && p.kind != DVIE_LOSS_MSE) {
      const float v = p.weight * g;
      p.grad[e] = p.beta ? p.grad[e] + v : v;
    }
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// cross entropy: logits a (B, C, H, W), target one-hot b; one thread per pixel
__global__ __launch_bounds__(RB) void ce_kernel(const dvie_loss_desc p) {
  __shared__ double sh[RB / 64];
  const float* a = (const float*)p.a;
  const float* b = (const float*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const long long npx = (long long)p.bsz * p.h * p.w;
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < npx;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / ((long long)p.w * p.h));
    int label = 0;
    float best = b[sb.at(n, 0, y, x)];
    float mx = a[sa.at(n, 0, y, x)];
    for (int c = 1; c < p.ch; ++c) {
      const float t = b[sb.at(n, c, y, x)];
      if (t > best) {
        best = t;
        label = c;
      }
      mx = fmaxf(mx, a[sa.at(n, c, y, x)]);
    }
    float s = 0.f;
    for (int c = 0; c < p.ch; ++c) s += expf(a[sa.at(n, c, y, x)] - mx);
    const float lse = mx + logf(s);
    acc += (double)(lse - a[sa.at(n, label, y, x)]);
    if (p.grad) {
      const float inv = p.weight / (float)npx;
      for (int c = 0; c < p.ch; ++c) {
        const float pr = expf(a[sa.at(n, c, y, x)] - mx) / s;
        const float v = (pr - (c == label ? 1.f : 0.f)) * inv;
        const long long gi = (((long long)n * p.ch + c) * p.h + y) * p.w + x;
        p.grad[gi] = p.beta ? p.grad[gi] + v : v;
      }
    }
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// mean |a - b| over two equally shaped strided tensors, channel fastest
template <typename T>
__global__ __launch_bounds__(RB) void l1nhwc_kernel(const dvie_loss_desc p) {
  __shared__ double sh[RB / 64];
  const T* a = (const T*)p.a;
  const T* b = (const T*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const long long tot = (long long)p.bsz * p.ch * p.h * p.w;
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % p.ch);
    const long long pix = e / p.ch;
    const int x = (int)(pix % p.w);
    const int y = (int)((pix / p.w) % p.h);
    const int n = (int)(pix / ((long long)p.w * p.h));
    float av, bv;
    if constexpr (sizeof(T) == 2) {
      av = bf2f(a[sa.at(n, c, y, x)]);
      bv = bf2f(b[sb.at(n, c, y, x)]);
    } else {
      av = a[sa.at(n, c, y, x)];
      bv = b[sb.at(n, c, y, x)];
    }
    acc += fabsf(av - bv);
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// the same feature L1 over dense bf16 NHWC rows (channel stride 1, pixel rows back to back,
// ch and the pixel stride multiples of 8): one 16-byte load of each map per 8 channels, the
// 8 differences summed in fp32 (exact inputs, 8 terms) and carried in double as above;
// one division per 8 elements instead of four per element
__global__ __launch_bounds__(RB) void l1nhwc8_kernel(const dvie_loss_desc p) {
  __shared__ double sh[RB / 64];
  const bf16_t* a = (const bf16_t*)p.a;
  const bf16_t* b = (const bf16_t*)p.b;
  const int nck = p.ch / 8;
  const long long tot = (long long)p.bsz * p.h * p.w * nck;
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / nck;
    const int k = (int)(e - q * nck);
    const i32x4 va = *(const i32x4*)(a + q * p.a_sw + 8 * k);
    const i32x4 vb = *(const i32x4*)(b + q * p.b_sw + 8 * k);
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned ua = (unsigned)va[i], ub = (unsigned)vb[i];
      t += fabsf(__uint_as_float(ua << 16) - __uint_as_float(ub << 16));
      t += fabsf(__uint_as_float(ua & 0xFFFF0000u) - __uint_as_float(ub & 0xFFFF0000u));
    }
    acc += (double)t;
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// mean over pixels of cos(a_pix, b_pix) over the channel axis (VGGCosineLoss,
// losses.py:182-207: a / sqrt(sum_c a^2) . b / sqrt(sum_c b^2), summed over channels).
// A group of L lanes (a power of two) owns one pixel and strides over its channels, so a
// wave reads 64/L neighbouring pixels' channel runs; the L partial sums meet by xor
// shuffles.  dot / (sqrt(saa) * sqrt(sbb)) is NaN for an all-zero feature vector, as the
// reference's 0/0 is.
template <typename T>
__global__ __launch_bounds__(RB) void cosnhwc_kernel(const dvie_loss_desc p, int L) {
  __shared__ double sh[RB / 64];
  const T* a = (const T*)p.a;
  const T* b = (const T*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const long long npx = (long long)p.bsz * p.h * p.w;
  const int lane = threadIdx.x & 63, sub = lane & (L - 1);
  const long long groups_per_block = RB / L;
  const long long g0 = (long long)blockIdx.x * groups_per_block + threadIdx.x / L;
  const long long gstride = (long long)gridDim.x * groups_per_block;
  double acc = 0.0;
  for (long long pix = g0; pix - threadIdx.x / L < npx; pix += gstride) {  // uniform trip count per wave
    float dot = 0.f, saa = 0.f, sbb = 0.f;
    const bool live = pix < npx;
    if (live) {
      const int x = (int)(pix % p.w);
      const int y = (int)((pix / p.w) % p.h);
      const int n = (int)(pix / ((long long)p.w * p.h));
      for (int c = sub; c < p.ch; c += L) {
        float av, bv;
        if constexpr (sizeof(T) == 2) {
          av = bf2f(a[sa.at(n, c, y, x)]);
          bv = bf2f(b[sb.at(n, c, y, x)]);
        } else {
          av = a[sa.at(n, c, y, x)];
          bv = b[sb.at(n, c, y, x)];
        }
        dot += av * bv;
        saa += av * av;
        sbb += bv * bv;
      }
    }
    for (int o = 1; o < L; o <<= 1) {
      dot += __shfl_xor(dot, o, 64);
      saa += __shfl_xor(saa, o, 64);
      sbb += __shfl_xor(sbb, o, 64);
    }
    if (live && sub == 0) acc += (double)(dot / (sqrtf(saa) * sqrtf(sbb)));
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// pixel accuracy of two label maps (IoU, losses.py:122-131: sum(pred == gt) / (B*H*W)).
// DVIE_LOSS_IOU: a, b are int64 (B, H, W) maps (strides sn, sh, sw; sc unused).
// DVIE_LOSS_ARGMAX_IOU: a, b are fp32 (B, C, H, W) scores; each pixel's label is its
// first maximal channel (torch.argmax), as validate's IoU(argmax(seg), argmax(gt_seg)).
__global__ __launch_bounds__(RB) void iou_kernel(const dvie_loss_desc p) {
  __shared__ double sh[RB / 64];
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const long long npx = (long long)p.bsz * p.h * p.w;
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < npx;
       e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % p.w);
    const int y = (int)((e / p.w) % p.h);
    const int n = (int)(e / ((long long)p.w * p.h));
    long long la, lb;
    if (p.kind == DVIE_LOSS_IOU) {
      la = ((const long long*)p.a)[sa.at(n, 0, y, x)];
      lb = ((const long long*)p.b)[sb.at(n, 0, y, x)];
    } else {
      const float* a = (const float*)p.a;
      const float* b = (const float*)p.b;
      float ba = a[sa.at(n, 0, y, x)], bb = b[sb.at(n, 0, y, x)];
      la = lb = 0;
      for (int c = 1; c < p.ch; ++c) {
        const float ta = a[sa.at(n, c, y, x)], tb = b[sb.at(n, c, y, x)];
        if (ta > ba || (ta != ta && ba == ba)) {  // torch.argmax: NaN is the maximum
          ba = ta;
          la = c;
        }
        if (tb > bb || (tb != tb && bb == bb)) {
          bb = tb;
          lb = c;
        }
      }
    }
    acc += la == lb ? 1.0 : 0.0;
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) p.partial[blockIdx.x] = t;
}

// ---------------- SSIM ----------------
constexpr int ST = 16;        // output tile edge
constexpr int SR = 5;         // window radius
constexpr int SE = ST + 2 * SR;

__device__ __forceinline__ void gauss11(float* g) {
  float s = 0.f;
  for (int i = 0; i < 11; ++i) {
    g[i] = expf(-(float)((i - 5) * (i - 5)) / 4.5f);
    s += g[i];
  }
  for (int i = 0; i < 11; ++i) g[i] /= s;
}

// forward: per-pixel ssim, partial sums, and (if grad) the three adjoint maps
// alpha = dL/dmu1, beta = dL/dE11, gamma = dL/dE12 into ws
__global__ __launch_bounds__(256) void ssim_fwd_kernel(const dvie_loss_desc p) {
  __shared__ float g[11];
  __shared__ float t1[SE][SE], t2[SE][SE];
  __shared__ float hs[5][SE][ST];
  __shared__ double sh[4];
  const float* a = (const float*)p.a;
  const float* b = (const float*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const int tid = threadIdx.x;
  const int tx = tid % ST, ty = tid / ST;
  const int plane = blockIdx.z;
  const int n = plane / p.ch, c = plane % p.ch;
  const int x0 = blockIdx.x * ST, y0 = blockIdx.y * ST;
  if (tid == 0) gauss11(g);
  for (int i = tid; i < SE * SE; i += 256) {
    const int yy = i / SE, xx = i % SE;
    const int gy = y0 + yy - SR, gx = x0 + xx - SR;
    float va = 0.f, vb = 0.f;
    if (gy >= 0 && gy < p.h && gx >= 0 && gx < p.w) {
      va = a[sa.at(n, c, gy, gx)];
      vb = b[sb.at(n, c, gy, gx)];
    }
    t1[yy][xx] = va;
    t2[yy][xx] = vb;
  }
  __syncthreads();
  for (int i = tid; i < SE * ST; i += 256) {
    const int yy = i / ST, xx = i % ST;
    float s1 = 0.f, s2 = 0.f, s11 = 0.f, s22 = 0.f, s12 = 0.f;
    for (int k = 0; k < 11; ++k) {
      const float u = t1[yy][xx + k], v = t2[yy][xx + k], w = g[k];
      s1 += w * u;
      s2 += w * v;
      s11 += w * u * u;
      s22 += w * v * v;
      s12 += w * u * v;
    }
    hs[0][yy][xx] = s1;
    hs[1][yy][xx] = s2;
    hs[2][yy][xx] = s11;
    hs[3][yy][xx] = s22;
    hs[4][yy][xx] = s12;
  }
  __syncthreads();
  float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
  for (int k = 0; k < 11; ++k) {
    const float w = g[k];
    m1 += w * hs[0][ty + k][tx];
    m2 += w * hs[1][ty + k][tx];
    e11 += w * hs[2][ty + k][tx];
    e22 += w * hs[3][ty + k][tx];
    e12 += w * hs[4][ty + k][tx];
  }
  const int oy = y0 + ty, ox = x0 + tx;
  double acc = 0.0;
  if (oy < p.h && ox < p.w) {
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    const float s11 = e11 - m1 * m1, s22 = e22 - m2 * m2, s12 = e12 - m1 * m2;
    const float A = 2.f * m1 * m2 + C1, B = 2.f * s12 + C2;
    const float Cc = m1 * m1 + m2 * m2 + C1, D = s11 + s22 + C2;
    const float Q = 1.f / (Cc * D);
    const float S = (A * B) * Q;
    acc = S;
    if (p.grad) {
      // derivatives written without dividing by A or B (either can cross zero: means of
      // opposite sign, negative covariance), as autograd differentiates num / den
      const float inv = -1.f / ((float)p.bsz * p.ch * p.h * p.w);
      const float dm1 = 2.f * Q * (m2 * (B - A) + m1 * S * (Cc - D));
      const float de11 = -S / D;
      const float de12 = 2.f * A * Q;
      const long long plane_sz = (long long)p.h * p.w;
      const long long np = (long long)p.bsz * p.ch * plane_sz;
      const long long idx = (long long)plane * plane_sz + (long long)oy * p.w + ox;
      p.ws[idx] = inv * dm1;
      p.ws[np + idx] = inv * de11;
      p.ws[2 * np + idx] = inv * de12;
    }
  }
  const double t = block_sum(acc, sh);
  if (tid == 0) p.partial[((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = t;
}

// backward: dx1 = G*alpha + 2 x1 (G*beta) + x2 (G*gamma)
__global__ __launch_bounds__(256) void ssim_bwd_kernel(const dvie_loss_desc p) {
  __shared__ float g[11];
  __shared__ float t[3][SE][SE];
  __shared__ float hs[3][SE][ST];
  const float* a = (const float*)p.a;
  const float* b = (const float*)p.b;
  const Shape sa{p.a_sn, p.a_sc, p.a_sh, p.a_sw}, sb{p.b_sn, p.b_sc, p.b_sh, p.b_sw};
  const int tid = threadIdx.x;
  const int tx = tid % ST, ty = tid / ST;
  const int plane = blockIdx.z;
  const int n = plane / p.ch, c = plane % p.ch;
  const int x0 = blockIdx.x * ST, y0 = blockIdx.y * ST;
  const long long plane_sz = (long long)p.h * p.w;
  const long long np = (long long)p.bsz * p.ch * plane_sz;
  if (tid == 0) gauss11(g);
  for (int i = tid; i < SE * SE; i += 256) {
    const int yy = i / SE, xx = i % SE;
    const int gy = y0 + yy - SR, gx = x0 + xx - SR;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (gy >= 0 && gy < p.h && gx >= 0 && gx < p.w) {
      const long long idx = (long long)plane * plane_sz + (long long)gy * p.w + gx;
      v0 = p.ws[idx];
      v1 = p.ws[np + idx];
      v2 = p.ws[2 * np + idx];
    }
    t[0][yy][xx] = v0;
    t[1][yy][xx] = v1;
    t[2][yy][xx] = v2;
  }
  __syncthreads();
  for (int i = tid; i < SE * ST; i += 256) {
    const int yy = i / ST, xx = i % ST;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int k = 0; k < 11; ++k) {
      s0 += g[k] * t[0][yy][xx + k];
      s1 += g[k] * t[1][yy][xx + k];
      s2 += g[k] * t[2][yy][xx + k];
    }
    hs[0][yy][xx] = s0;
    hs[1][yy][xx] = s1;
    hs[2][yy][xx] = s2;
  }
  __syncthreads();
  float u0 = 0.f, u1 = 0.f, u2 = 0.f;
  for (int k = 0; k < 11; ++k) {
    u0 += g[k] * hs[0][ty + k][tx];
    u1 += g[k] * hs[1][ty + k][tx];
    u2 += g[k] * hs[2][ty + k][tx];
  }
  const int oy = y0 + ty, ox = x0 + tx;
  if (oy < p.h && ox < p.w) {
    const float x1 = a[sa.at(n, c, oy, ox)], x2 = b[sb.at(n, c, oy, ox)];
    const float v = p.weight * (u0 + 2.f * x1 * u1 + x2 * u2);
    const long long gi = (long long)plane * plane_sz + (long long)oy * p.w + ox;
    p.grad[gi] = p.beta ? p.grad[gi] + v : v;
  }
}

// out[j] (+)= vscale * (sum of partials * mul + add)
__global__ __launch_bounds__(RB) void finalize_kernel(const double* part, int nb, int nout, float* out, double mul,
                                                      double add, float vscale, int acc) {
  __shared__ double sh[RB / 64];
  for (int j = 0; j < nout; ++j) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[(long long)j * nb + i];
    const double t = block_sum(s, sh);
    if (threadIdx.x == 0) {
      const float v = vscale * (float)(t * mul + add);
      out[j] = acc ? out[j] + v : v;
    }
  }
}

// one workgroup: out[0] = x[0] + x[1] + ... in index order (lane 0 walks the terms)
__global__ __launch_bounds__(64) void sum_f32_kernel(const float* x, int n, float* out) {
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += x[i];
    out[0] = s;
  }
}

struct LossPlan {
  int blocks;       // partial count
  int per_sample;   // MSE: blocks per sample
  dim3 grid;
};

// lanes per pixel of the cosine kernel: the channel count rounded up to a power of two,
// capped at one wave
static int cos_lanes(int ch) {
  int L = 1;
  while (L < ch && L < 64) L <<= 1;
  return L;
}

static LossPlan plan_loss(const dvie_loss_desc& d) {
  LossPlan lp{};
  const long long px = (long long)d.bsz * d.h * d.w;
  const long long tot = px * d.ch;
  switch (d.kind) {
    case DVIE_LOSS_SSIM:
      lp.grid = dim3((d.w + ST - 1) / ST, (d.h + ST - 1) / ST, d.bsz * d.ch);
      lp.blocks = lp.grid.x * lp.grid.y * lp.grid.z;
      break;
    case DVIE_LOSS_MSE: {
      long long per = (long long)d.ch * d.h * d.w;
      int ps = (int)((per + RB * 8 - 1) / (RB * 8));
      if (ps > 256) ps = 256;
      if (ps < 1) ps = 1;
      lp.per_sample = ps;
      lp.blocks = ps * d.bsz;
      lp.grid = dim3(lp.blocks);
      break;
    }
    case DVIE_LOSS_COSNHWC: {
      long long b = (px * cos_lanes(d.ch) + RB * 8 - 1) / (RB * 8);
      lp.blocks = (int)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
      lp.grid = dim3(lp.blocks);
      break;
    }
    case DVIE_LOSS_IOU:
    case DVIE_LOSS_ARGMAX_IOU:
    case DVIE_LOSS_CE: {
      long long b = (px + RB * 4 - 1) / (RB * 4);
      lp.blocks = (int)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
      lp.grid = dim3(lp.blocks);
      break;
    }
    default: {
      long long b = (tot + RB * 8 - 1) / (RB * 8);
      lp.blocks = (int)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
      lp.grid = dim3(lp.blocks);
      break;
    }
  }
  return lp;
}

}  // namespace dvie

using namespace dvie;

extern "C" {

size_t dvie_loss_partial_count(const dvie_loss_desc* d) { return d ? (size_t)plan_loss(*d).blocks : 0; }

size_t dvie_loss_ws_floats(const dvie_loss_desc* d) {
  if (!d || d->kind != DVIE_LOSS_SSIM) return 0;
  return (size_t)3 * d->bsz * d->ch * d->h * d->w;
}

int dvie_loss(const dvie_loss_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->a && d->b && d->out && d->partial, "loss: null pointer");
  DVIE_CHECK_ARG(d->bsz > 0 && d->ch > 0 && d->h > 0 && d->w > 0, "loss: empty shape");
  if (d->kind == DVIE_LOSS_GDL) DVIE_CHECK_ARG(d->h > 1 && d->w > 1, "loss: GDL needs h,w > 1");
  if (d->kind == DVIE_LOSS_SSIM && d->grad) DVIE_CHECK_ARG(d->ws != nullptr, "loss: SSIM grad needs ws");
  if (d->kind >= DVIE_LOSS_COSNHWC)
    DVIE_CHECK_ARG(d->grad == nullptr, "loss: kind %d is a metric (no gradient)", d->kind);
  hipStream_t s = (hipStream_t)stream;
  const LossPlan lp = plan_loss(*d);
  const float vs = d->out_scale;
  const int acc = d->out_acc;
  const double px = (double)d->bsz * d->h * d->w;
  const double tot = px * d->ch;
  switch (d->kind) {
    case DVIE_LOSS_L1:
    case DVIE_LOSS_GDL:
      DVIE_LAUNCH(l1gdl_kernel, lp.grid, dim3(RB), 0, s, *d, 0);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out,
                         d->kind == DVIE_LOSS_L1 ? 1.0 / tot : 1.0, 0.0, vs, acc);
      break;
    case DVIE_LOSS_MSE:
      DVIE_LAUNCH(l1gdl_kernel, lp.grid, dim3(RB), 0, s, *d, lp.per_sample);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.per_sample, d->bsz, d->out,
                         1.0 / ((double)d->ch * d->h * d->w), 0.0, vs, acc);
      break;
    case DVIE_LOSS_CE:
      DVIE_LAUNCH(ce_kernel, lp.grid, dim3(RB), 0, s, *d);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out, 1.0 / px, 0.0, vs, acc);
      break;
    case DVIE_LOSS_SSIM:
      DVIE_LAUNCH(ssim_fwd_kernel, lp.grid, dim3(256), 0, s, *d);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out, -1.0 / tot,
                         1.0, vs, acc);
      if (d->grad) DVIE_LAUNCH(ssim_bwd_kernel, lp.grid, dim3(256), 0, s, *d);
      break;
    case DVIE_LOSS_L1NHWC:
      if (d->dtype == DVIE_BF16 && d->a_sc == 1 && d->b_sc == 1 && d->ch % 8 == 0 && d->a_sw % 8 == 0 &&
          d->b_sw % 8 == 0 && d->a_sh == (long long)d->w * d->a_sw && d->b_sh == (long long)d->w * d->b_sw &&
          d->a_sn == (long long)d->h * d->a_sh && d->b_sn == (long long)d->h * d->b_sh &&
          ((uintptr_t)d->a & 15) == 0 && ((uintptr_t)d->b & 15) == 0)
        DVIE_LAUNCH(l1nhwc8_kernel, lp.grid, dim3(RB), 0, s, *d);
      else if (d->dtype == DVIE_BF16)
        DVIE_LAUNCH(l1nhwc_kernel<bf16_t>, lp.grid, dim3(RB), 0, s, *d);
      else
        DVIE_LAUNCH(l1nhwc_kernel<float>, lp.grid, dim3(RB), 0, s, *d);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out, 1.0 / tot, 0.0, vs, acc);
      break;
    case DVIE_LOSS_COSNHWC:
      if (d->dtype == DVIE_BF16)
        DVIE_LAUNCH(cosnhwc_kernel<bf16_t>, lp.grid, dim3(RB), 0, s, *d, cos_lanes(d->ch));
      else
        DVIE_LAUNCH(cosnhwc_kernel<float>, lp.grid, dim3(RB), 0, s, *d, cos_lanes(d->ch));
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out,
                         (double)d->weight / px, 0.0, vs, acc);
      break;
    case DVIE_LOSS_IOU:
    case DVIE_LOSS_ARGMAX_IOU:
      DVIE_LAUNCH(iou_kernel, lp.grid, dim3(RB), 0, s, *d);
      DVIE_LAUNCH(finalize_kernel, dim3(1), dim3(RB), 0, s, d->partial, lp.blocks, 1, d->out, 1.0 / px, 0.0, vs, acc);
      break;
    default:
      DVIE_CHECK_ARG(false, "loss: unknown kind %d", d->kind);
  }
  DVIE_RETURN_LAUNCH();
}

int dvie_sum_f32(const float* x, int n, float* out, void* stream) {
  DVIE_CHECK_ARG(x && out && n > 0, "sum_f32: args");
  DVIE_LAUNCH(sum_f32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, x, n, out);
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"
