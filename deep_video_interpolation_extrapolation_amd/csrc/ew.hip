// NHWC pointwise kernels: multi-resolution fuse sums with bilinear upsampling
// (align_corners=False), the gather-form adjoint of that upsampling, 2x2 average pooling
// and its adjoint, copies, feature-L1 sign gradients and NCHW<->NHWC packing.  Every op
// shares the same epilogue (residual add, accumulate, activation, activation-derivative)
// so backward contributions fuse into one pass.  Each thread owns 4 channels of one pixel.
//
// Reference ops replaced: F.interpolate/F.upsample(mode='bilinear') of
// nets/HRNet.py:219-222,577-580 (+ the sums/LeakyReLU of l.212-225), AvgPool2d of
// nets/vgg.py:9, preprocess_norm of utils/net_utils.py:11-23, torch.cat of
// nets/HRNet.py:539,582 (by writing channel slices), and their autograd backward ops.
#include "common.h"

namespace dvie {

// torch area_pixel_compute_source_index (align_corners=False, non-cubic) + the
// neighbour/lambda selection of upsample_bilinear2d
struct Lerp {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lerp lerp_src(int dst, int in_size, int out_size) {
  const float scale = (float)in_size / (float)out_size;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  Lerp r;
  r.i0 = (int)src;
  if (r.i0 > in_size - 1) r.i0 = in_size - 1;
  r.i1 = r.i0 + ((r.i0 < in_size - 1) ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

template <typename T>
__device__ __forceinline__ f32x4 up_sample(const T* __restrict__ s, long long ld, int n, int y, int x, int c, int sh,
                                           int sw, int h, int w) {
  if (sh == h && sw == w) return V4<T>::load(s + (((long long)n * sh + y) * sw + x) * ld + c);
  const Lerp ly = lerp_src(y, sh, h), lx = lerp_src(x, sw, w);
  const long long r0 = ((long long)n * sh + ly.i0) * sw, r1 = ((long long)n * sh + ly.i1) * sw;
  const f32x4 a = V4<T>::load(s + (r0 + lx.i0) * ld + c);
  const f32x4 b = V4<T>::load(s + (r0 + lx.i1) * ld + c);
  const f32x4 cc = V4<T>::load(s + (r1 + lx.i0) * ld + c);
  const f32x4 d = V4<T>::load(s + (r1 + lx.i1) * ld + c);
  return ly.l0 * (lx.l0 * a + lx.l1 * b) + ly.l1 * (lx.l0 * cc + lx.l1 * d);
}

// weight of fine index `f` (fine size `fs`) onto coarse index `cidx` (coarse size `cs`)
__device__ __forceinline__ float upt_weight(int f, int cidx, int cs, int fs) {
  const Lerp l = lerp_src(f, cs, fs);
  float wgt = 0.f;
  if (l.i0 == cidx) wgt += l.l0;
  if (l.i1 == cidx) wgt += l.l1;
  return wgt;
}

template <typename T>
__global__ __launch_bounds__(256) void ew_kernel(const dvie_ew_desc p) {
  const int cq = p.c >> 2;
  const long long total = (long long)p.n * p.h * p.w * cq;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(e % cq);
    const long long pix = e / cq;
    const int x = (int)(pix % p.w);
    const int y = (int)((pix / p.w) % p.h);
    const int n = (int)(pix / ((long long)p.w * p.h));
    const int c = q * 4;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    switch (p.op) {
      case DVIE_EW_FUSE:
        v = up_sample<T>((const T*)p.src0, p.src_ld0, n, y, x, c, p.sh0, p.sw0, p.h, p.w);
        if (p.nsrc > 1) v += up_sample<T>((const T*)p.src1, p.src_ld1, n, y, x, c, p.sh1, p.sw1, p.h, p.w);
        if (p.nsrc > 2) v += up_sample<T>((const T*)p.src2, p.src_ld2, n, y, x, c, p.sh2, p.sw2, p.h, p.w);
        break;
      case DVIE_EW_UPT: {
        // coarse output (y, x) of a (h, w) grid, fine source (sh0, sw0)
        const T* s = (const T*)p.src0;
        const float fy = (float)p.sh0 / (float)p.h, fx = (float)p.sw0 / (float)p.w;
        int ylo = (int)floorf(((float)y - 0.5f) * fy - 0.5f) - 1, yhi = (int)ceilf(((float)y + 1.5f) * fy) + 1;
        int xlo = (int)floorf(((float)x - 0.5f) * fx - 0.5f) - 1, xhi = (int)ceilf(((float)x + 1.5f) * fx) + 1;
        if (ylo < 0) ylo = 0;
        if (xlo < 0) xlo = 0;
        if (yhi > p.sh0 - 1) yhi = p.sh0 - 1;
        if (xhi > p.sw0 - 1) xhi = p.sw0 - 1;
        for (int Y = ylo; Y <= yhi; ++Y) {
          const float wy = upt_weight(Y, y, p.h, p.sh0);
          if (wy == 0.f) continue;
          f32x4 row = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int X = xlo; X <= xhi; ++X) {
            const float wx = upt_weight(X, x, p.w, p.sw0);
            if (wx == 0.f) continue;
            row += wx * V4<T>::load(s + (((long long)n * p.sh0 + Y) * p.sw0 + X) * p.src_ld0 + c);
          }
          v += wy * row;
        }
        break;
      }
      case DVIE_EW_POOL: {
        const T* s = (const T*)p.src0;
        const long long r0 = ((long long)n * p.sh0 + 2 * y) * p.sw0 + 2 * x;
        const long long r1 = r0 + p.sw0;
        v = V4<T>::load(s + r0 * p.src_ld0 + c) + V4<T>::load(s + (r0 + 1) * p.src_ld0 + c) +
            V4<T>::load(s + r1 * p.src_ld0 + c) + V4<T>::load(s + (r1 + 1) * p.src_ld0 + c);
        v = v / 4.f;
        break;
      }
      case DVIE_EW_POOLT: {
        const T* s = (const T*)p.src0;
        v = V4<T>::load(s + (((long long)n * p.sh0 + (y >> 1)) * p.sw0 + (x >> 1)) * p.src_ld0 + c) / 4.f;
        break;
      }
      case DVIE_EW_COPY:
        v = V4<T>::load((const T*)p.src0 + pix * p.src_ld0 + c);
        break;
      case DVIE_EW_L1SIGN: {
        const f32x4 a = V4<T>::load((const T*)p.src0 + pix * p.src_ld0 + c);
        const f32x4 b = V4<T>::load((const T*)p.src1 + pix * p.src_ld1 + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float d = a[k] - b[k];
          v[k] = d > 0.f ? p.scale : (d < 0.f ? -p.scale : 0.f);
        }
        break;
      }
      case DVIE_EW_NCHW: {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ch = c + k;
          if (ch < p.ext_c) {
            float t = p.ext[(long long)n * p.sn + (long long)ch * p.sc + (long long)y * p.sh + (long long)x * p.sw];
            if (p.mean) t = (t - p.mean[ch]) / p.std[ch];
            v[k] = t;
          }
        }
        break;
      }
      case DVIE_EW_TONCHW: {
        const f32x4 a = V4<T>::load((const T*)p.src0 + pix * p.src_ld0 + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ch = c + k;
          if (ch < p.ext_c) {
            float* d = p.ext + (long long)n * p.sn + (long long)ch * p.sc + (long long)y * p.sh + (long long)x * p.sw;
            const float v = p.std ? a[k] / p.std[ch] : a[k];  // adjoint of preprocess_norm
            *d = p.beta ? *d + v : v;
          }
        }
        continue;
      }
      default:
        break;
    }
    T* yp = (T*)p.y + pix * p.y_ld + c;
    if (p.res) v += V4<T>::load((const T*)p.res + pix * p.res_ld + c);
    if (p.beta) v += V4<T>::load(yp);
    if (p.act) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      const f32x4 z = V4<T>::load((const T*)p.z + pix * p.z_ld + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] *= act_dz(z[k], p.dact, p.alpha);
    }
    V4<T>::store(yp, v);
  }
}

}  // namespace dvie

using namespace dvie;

extern "C" int dvie_ew(const dvie_ew_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->c > 0 && d->c % 4 == 0, "ew: c=%d must be a multiple of 4", d ? d->c : -1);
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0, "ew: empty shape");
  DVIE_CHECK_ARG(d->op == DVIE_EW_TONCHW || (d->y && d->y_ld % 4 == 0), "ew: y");
  if (d->op == DVIE_EW_POOL) DVIE_CHECK_ARG(d->sh0 == 2 * d->h && d->sw0 == 2 * d->w, "ew: pool shape");
  if (d->op == DVIE_EW_POOLT) DVIE_CHECK_ARG(d->h == 2 * d->sh0 && d->w == 2 * d->sw0, "ew: poolT shape");
  if (d->op == DVIE_EW_NCHW || d->op == DVIE_EW_TONCHW) DVIE_CHECK_ARG(d->ext != nullptr, "ew: ext");
  if (d->dact) DVIE_CHECK_ARG(d->z != nullptr && d->z_ld % 4 == 0, "ew: z");
  const long long total = (long long)d->n * d->h * d->w * (d->c / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == DVIE_BF16)
    hipLaunchKernelGGL(ew_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, *d);
  else
    hipLaunchKernelGGL(ew_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, *d);
  DVIE_RETURN_LAUNCH();
}
