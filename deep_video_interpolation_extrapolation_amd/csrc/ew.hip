// NHWC pointwise kernels: multi-resolution fuse sums with bilinear upsampling
// (align_corners False or True), the gather-form adjoint of that upsampling, 2x2 average pooling
// and its adjoint, copies, feature-L1 sign gradients and NCHW<->NHWC packing.  Every op
// shares the same epilogue (residual add, accumulate, activation, activation-derivative)
// so backward contributions fuse into one pass.  Each thread owns 8 (bf16, 16-byte
// accesses) or 4 channels of one pixel; blocks run along one image row.
//
// Reference ops replaced: F.interpolate/F.upsample(mode='bilinear') of
// nets/HRNet.py:219-222,577-580 (+ the sums/LeakyReLU of l.212-225), AvgPool2d of
// nets/vgg.py:9, preprocess_norm of utils/net_utils.py:11-23, torch.cat of
// nets/HRNet.py:539,582 (by writing channel slices), and their autograd backward ops.
#include <stdlib.h>

#include "common.h"

namespace dvie {

// torch area_pixel_compute_source_index (non-cubic) + the neighbour/lambda selection of
// upsample_bilinear2d; align_corners=True maps the corner pixels onto each other
struct Lerp {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lerp lerp_src(int dst, int in_size, int out_size, int align) {
  float src;
  if (align) {
    const float scale = out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.f;
    src = scale * (float)dst;
  } else {
    const float scale = (float)in_size / (float)out_size;
    src = scale * ((float)dst + 0.5f) - 0.5f;
  }
  if (src < 0.f) src = 0.f;
  Lerp r;
  r.i0 = (int)src;
  if (r.i0 > in_size - 1) r.i0 = in_size - 1;
  r.i1 = r.i0 + ((r.i0 < in_size - 1) ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

typedef __bf16 ew_bf16x2 __attribute__((ext_vector_type(2)));
typedef float ew_f32x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32; = f2bf for every
// non-NaN input, a quiet NaN for NaN)
__device__ __forceinline__ uint32_t ew_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((ew_f32x2{a, b}), ew_bf16x2));
}

// VW-channel vectors (16 B for bf16 x8 / fp32 x4; 8 B for bf16 x4)
template <typename T, int VW>
struct VecN;
template <>
struct VecN<bf16_t, 8> {
  __device__ __forceinline__ static void load(const bf16_t* p, float* v) {
    const i32x4 r = *(const i32x4*)p;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(((uint32_t)r[k]) << 16);
      v[2 * k + 1] = __uint_as_float(((uint32_t)r[k]) & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float* v) {
    i32x4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = (int)ew_pack(v[2 * k], v[2 * k + 1]);
    *(i32x4*)p = r;
  }
};
template <typename T>
struct VecN<T, 4> {
  __device__ __forceinline__ static void load(const T* p, float* v) {
    const f32x4 r = V4<T>::load(p);
    v[0] = r[0];
    v[1] = r[1];
    v[2] = r[2];
    v[3] = r[3];
  }
  __device__ __forceinline__ static void store(T* p, const float* v) { V4<T>::store(p, f32x4{v[0], v[1], v[2], v[3]}); }
};

template <typename T, int VW>
__device__ __forceinline__ void up_sample_add(float* v, const T* __restrict__ s, long long ld, int n, int y, int x,
                                              int c, int sh, int sw, int h, int w, int align) {
  float t[VW];
  if (sh == h && sw == w) {
    VecN<T, VW>::load(s + (((long long)n * sh + y) * sw + x) * ld + c, t);
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] += t[k];
    return;
  }
  const Lerp ly = lerp_src(y, sh, h, align), lx = lerp_src(x, sw, w, align);
  const long long r0 = ((long long)n * sh + ly.i0) * sw, r1 = ((long long)n * sh + ly.i1) * sw;
  float a[VW], b[VW], cc[VW], d[VW];
  VecN<T, VW>::load(s + (r0 + lx.i0) * ld + c, a);
  VecN<T, VW>::load(s + (r0 + lx.i1) * ld + c, b);
  VecN<T, VW>::load(s + (r1 + lx.i0) * ld + c, cc);
  VecN<T, VW>::load(s + (r1 + lx.i1) * ld + c, d);
#pragma unroll
  for (int k = 0; k < VW; ++k) v[k] += ly.l0 * (lx.l0 * a[k] + lx.l1 * b[k]) + ly.l1 * (lx.l0 * cc[k] + lx.l1 * d[k]);
}

// weight of fine index `f` (fine size `fs`) onto coarse index `cidx` (coarse size `cs`)
__device__ __forceinline__ float upt_weight(int f, int cidx, int cs, int fs, int align) {
  const Lerp l = lerp_src(f, cs, fs, align);
  float wgt = 0.f;
  if (l.i0 == cidx) wgt += l.l0;
  if (l.i1 == cidx) wgt += l.l1;
  return wgt;
}

// Upsample adjoint for an integer ratio R (align_corners False): the fine rows / columns whose
// stencil can reach coarse index i are R*i - R/2 - 1 .. R*i + R + R/2 (2R + 2 candidates, one
// spare on each side).  Row weights are uniform over a block (one coarse row), so zero rows
// are skipped by a uniform branch; within a row every candidate column is loaded
// unconditionally (clamped address, zero weight outside), so the 2R + 2 loads of a row issue
// back to back instead of one per divergent branch.  Weights: the forward's own lerp.
template <typename T, int VW, int R>
__device__ __forceinline__ void upt_ratio(float* v, const T* __restrict__ s, long long ld, int n, int y, int x, int c,
                                          int h, int w, int sh, int sw) {
  constexpr int NC = 2 * R + 2;
  const int Y0 = R * y - R / 2 - 1, X0 = R * x - R / 2 - 1;
  float wx[NC];
  int xo[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int X = X0 + j;
    const bool in = X >= 0 && X < sw;
    wx[j] = in ? upt_weight(X, x, w, sw, 0) : 0.f;
    xo[j] = in ? X : 0;
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int Y = Y0 + i;
    if (Y < 0 || Y >= sh) continue;
    const float wy = upt_weight(Y, y, h, sh, 0);
    if (wy == 0.f) continue;
    const T* srow = s + ((long long)n * sh + Y) * sw * ld + c;
    if constexpr (VW == 8) {  // bf16: keep the loads packed (4 VGPRs each) until their FMAs
      i32x4 raw[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) raw[j] = *(const i32x4*)(srow + (long long)xo[j] * ld);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const float wgt = wy * wx[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += wgt * __uint_as_float(((uint32_t)raw[j][k]) << 16);
          v[2 * k + 1] += wgt * __uint_as_float(((uint32_t)raw[j][k]) & 0xffff0000u);
        }
      }
    } else {
      float t[NC][VW];
#pragma unroll
      for (int j = 0; j < NC; ++j) VecN<T, VW>::load(srow + (long long)xo[j] * ld, t[j]);
#pragma unroll
      for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int k = 0; k < VW; ++k) v[k] += wy * wx[j] * t[j][k];
    }
  }
}

// One thread = VW channels of one pixel; blockIdx.y = image row (n, y), so the per-element
// index math is one 32-bit division by the channel-vector count.
// OPK >= 0: the kernel is specialised to that op (the others compile away), so the hot
// multi-resolution ops do not carry the register allocation of the largest case; -1: any op;
// -2: any op but the upsample adjoint.
template <typename T, int VW, int OPK>
__global__ __launch_bounds__(256) void ew_kernel(const dvie_ew_desc p, int cq) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= p.w * cq) return;
  const int x = e / cq;
  const int c = (e - x * cq) * VW;
  const int row = blockIdx.y;
  const int n = row / p.h, y = row - (row / p.h) * p.h;
  const long long pix = (long long)row * p.w + x;
  float v[VW];
#pragma unroll
  for (int k = 0; k < VW; ++k) v[k] = 0.f;
  switch (OPK >= 0 ? OPK : p.op) {
    case DVIE_EW_FUSE:
      up_sample_add<T, VW>(v, (const T*)p.src0, p.src_ld0, n, y, x, c, p.sh0, p.sw0, p.h, p.w, p.align);
      if (p.nsrc > 1)
        up_sample_add<T, VW>(v, (const T*)p.src1, p.src_ld1, n, y, x, c, p.sh1, p.sw1, p.h, p.w, p.align);
      if (p.nsrc > 2)
        up_sample_add<T, VW>(v, (const T*)p.src2, p.src_ld2, n, y, x, c, p.sh2, p.sw2, p.h, p.w, p.align);
      break;
    case DVIE_EW_UPT: {
      if constexpr (OPK == -2) break;  // (launched through its own instance)
      // coarse output (y, x) of a (h, w) grid, fine source (sh0, sw0)
      const T* s = (const T*)p.src0;
      if (!p.align && p.sh0 == 2 * p.h && p.sw0 == 2 * p.w) {
        upt_ratio<T, VW, 2>(v, s, p.src_ld0, n, y, x, c, p.h, p.w, p.sh0, p.sw0);
        break;
      }
      if (!p.align && p.sh0 == 4 * p.h && p.sw0 == 4 * p.w) {
        upt_ratio<T, VW, 4>(v, s, p.src_ld0, n, y, x, c, p.h, p.w, p.sh0, p.sw0);
        break;
      }
      // fine rows/cols whose bilinear stencil can touch coarse (y, x), widened by one
      const float fy = p.align ? (float)(p.sh0 - 1) / (float)max(p.h - 1, 1) : (float)p.sh0 / (float)p.h;
      const float fx = p.align ? (float)(p.sw0 - 1) / (float)max(p.w - 1, 1) : (float)p.sw0 / (float)p.w;
      int ylo = (int)floorf(((float)y - 1.f) * fy - 0.5f) - 1, yhi = (int)ceilf(((float)y + 1.5f) * fy) + 1;
      int xlo = (int)floorf(((float)x - 1.f) * fx - 0.5f) - 1, xhi = (int)ceilf(((float)x + 1.5f) * fx) + 1;
      if (ylo < 0) ylo = 0;
      if (xlo < 0) xlo = 0;
      if (yhi > p.sh0 - 1) yhi = p.sh0 - 1;
      if (xhi > p.sw0 - 1) xhi = p.sw0 - 1;
      for (int Y = ylo; Y <= yhi; ++Y) {
        const float wy = upt_weight(Y, y, p.h, p.sh0, p.align);
        if (wy == 0.f) continue;
        float rowv[VW];
#pragma unroll
        for (int k = 0; k < VW; ++k) rowv[k] = 0.f;
        for (int X = xlo; X <= xhi; ++X) {
          const float wx = upt_weight(X, x, p.w, p.sw0, p.align);
          if (wx == 0.f) continue;
          float t[VW];
          VecN<T, VW>::load(s + (((long long)n * p.sh0 + Y) * p.sw0 + X) * p.src_ld0 + c, t);
#pragma unroll
          for (int k = 0; k < VW; ++k) rowv[k] += wx * t[k];
        }
#pragma unroll
        for (int k = 0; k < VW; ++k) v[k] += wy * rowv[k];
      }
      break;
    }
    case DVIE_EW_POOL: {
      const T* s = (const T*)p.src0;
      const long long r0 = ((long long)n * p.sh0 + 2 * y) * p.sw0 + 2 * x;
      const long long r1 = r0 + p.sw0;
      float a[VW], b[VW], cc[VW], d[VW];
      VecN<T, VW>::load(s + r0 * p.src_ld0 + c, a);
      VecN<T, VW>::load(s + (r0 + 1) * p.src_ld0 + c, b);
      VecN<T, VW>::load(s + r1 * p.src_ld0 + c, cc);
      VecN<T, VW>::load(s + (r1 + 1) * p.src_ld0 + c, d);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] = (a[k] + b[k] + cc[k] + d[k]) / 4.f;
      break;
    }
    case DVIE_EW_POOLT: {
      const T* s = (const T*)p.src0;
      VecN<T, VW>::load(s + (((long long)n * p.sh0 + (y >> 1)) * p.sw0 + (x >> 1)) * p.src_ld0 + c, v);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] = v[k] / 4.f;
      break;
    }
    case DVIE_EW_COPY:
      VecN<T, VW>::load((const T*)p.src0 + pix * p.src_ld0 + c, v);
      break;
    case DVIE_EW_IM2COL: {
      const int t = c / p.ext_c, ch = c - t * p.ext_c;
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] = 0.f;
      if (t < p.sh0 * p.sw0) {
        const int ty = t / p.sw0, tx = t - ty * p.sw0;
        const int Y = y + p.sh1 + ty * p.sh2, X = x + p.sw1 + tx * p.sw2;
        if (Y >= 0 && Y < p.h && X >= 0 && X < p.w)
          VecN<T, VW>::load((const T*)p.src0 + (((long long)n * p.h + Y) * p.w + X) * p.src_ld0 + ch, v);
      }
      break;
    }
    case DVIE_EW_L1SIGN: {
      float a[VW], b[VW];
      VecN<T, VW>::load((const T*)p.src0 + pix * p.src_ld0 + c, a);
      VecN<T, VW>::load((const T*)p.src1 + pix * p.src_ld1 + c, b);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        const float d = a[k] - b[k];
        v[k] = d > 0.f ? p.scale : (d < 0.f ? -p.scale : 0.f);
      }
      break;
    }
    case DVIE_EW_NCHW: {
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        const int ch = c + k;
        if (ch < p.ext_c) {
          const bool second = p.src1 != nullptr && ch >= p.sh1;
          const float* e = second ? (const float*)p.src1 : p.ext;
          const int cc = second ? ch - p.sh1 : ch;
          float t = e[(long long)n * p.sn + (long long)cc * p.sc + (long long)y * p.sh + (long long)x * p.sw];
          if (p.mean) t = (t - p.mean[ch]) / p.std[ch];
          v[k] = t;
        }
      }
      break;
    }
    case DVIE_EW_MASK: {
      const float m = p.ext[(long long)n * p.sn + (long long)y * p.sh + (long long)x * p.sw];
      const float f = p.ext_c ? 1.f - m : m;
      VecN<T, VW>::load((const T*)p.src0 + pix * p.src_ld0 + c, v);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] *= f;
      break;
    }
    case DVIE_EW_TONCHW: {
      float a[VW];
      VecN<T, VW>::load((const T*)p.src0 + pix * p.src_ld0 + c, a);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        const int ch = c + k;
        if (ch < p.ext_c) {
          float* d = p.ext + (long long)n * p.sn + (long long)ch * p.sc + (long long)y * p.sh + (long long)x * p.sw;
          const float t = p.std ? a[k] / p.std[ch] : a[k];  // adjoint of preprocess_norm
          *d = p.beta ? *d + t : t;
        }
      }
      return;
    }
    default:
      break;
  }
  T* yp = (T*)p.y + pix * p.y_ld + c;
  float t[VW];
  if (p.res) {
    VecN<T, VW>::load((const T*)p.res + pix * p.res_ld + c, t);
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] += t[k];
  }
  if (p.beta) {
    VecN<T, VW>::load(yp, t);
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] += t[k];
  }
  if (p.act) {
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
  }
  if (p.dact) {
    VecN<T, VW>::load((const T*)p.z + pix * p.z_ld + c, t);
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] *= act_dz(t[k], p.dact, p.alpha);
  }
  VecN<T, VW>::store(yp, v);
}

// EW_FUSE with two horizontally adjacent output pixels per thread (bf16 x8).  For an
// upsampled source the pair's bilinear columns are {i0, i1} of the left pixel plus the right
// pixel's i1 (its i0 is one of the left pixel's: the source step per output pixel is <= 1), so
// a source costs 2 rows x 3 column loads per pair instead of 2 x 4 per pixel; at 4x the pair
// shares both columns.  Same lerp arithmetic and summation order as ew_kernel.
template <typename T, int VW>
__global__ __launch_bounds__(256) void ew_fuse2_kernel(const dvie_ew_desc p, int cq) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int wp = (p.w + 1) >> 1;
  if (e >= wp * cq) return;
  const int xp = e / cq;
  const int c = (e - xp * cq) * VW;
  const int x = 2 * xp;
  const bool two = x + 1 < p.w;
  const int row = blockIdx.y;
  const int n = row / p.h, y = row - (row / p.h) * p.h;
  float v0[VW], v1[VW];
#pragma unroll
  for (int k = 0; k < VW; ++k) v0[k] = v1[k] = 0.f;
  auto src_add = [&](const T* s, long long ld, int sh, int sw) {
    float a[VW], b[VW];
    if (sh == p.h && sw == p.w) {
      VecN<T, VW>::load(s + (((long long)n * sh + y) * sw + x) * ld + c, a);
      VecN<T, VW>::load(s + (((long long)n * sh + y) * sw + (two ? x + 1 : x)) * ld + c, b);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        v0[k] += a[k];
        v1[k] += b[k];
      }
      return;
    }
    const Lerp ly = lerp_src(y, sh, p.h, p.align);
    const Lerp l0 = lerp_src(x, sw, p.w, p.align), l1 = lerp_src(two ? x + 1 : x, sw, p.w, p.align);
    const long long r0 = ((long long)n * sh + ly.i0) * sw, r1 = ((long long)n * sh + ly.i1) * sw;
    // columns: c0 = l0.i0, c1 = l0.i1, c2 = l1.i1; the right pixel's i0 is c0 or c1
    const bool rsh = l1.i0 != l0.i0;  // right pixel starts at c1
    float t00[VW], t01[VW], t02[VW], t10[VW], t11[VW], t12[VW];
    VecN<T, VW>::load(s + (r0 + l0.i0) * ld + c, t00);
    VecN<T, VW>::load(s + (r0 + l0.i1) * ld + c, t01);
    VecN<T, VW>::load(s + (r0 + l1.i1) * ld + c, t02);
    VecN<T, VW>::load(s + (r1 + l0.i0) * ld + c, t10);
    VecN<T, VW>::load(s + (r1 + l0.i1) * ld + c, t11);
    VecN<T, VW>::load(s + (r1 + l1.i1) * ld + c, t12);
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      v0[k] += ly.l0 * (l0.l0 * t00[k] + l0.l1 * t01[k]) + ly.l1 * (l0.l0 * t10[k] + l0.l1 * t11[k]);
      const float ra = rsh ? t01[k] : t00[k], rb = t02[k];
      const float rc = rsh ? t11[k] : t10[k], rd = t12[k];
      v1[k] += ly.l0 * (l1.l0 * ra + l1.l1 * rb) + ly.l1 * (l1.l0 * rc + l1.l1 * rd);
    }
  };
  src_add((const T*)p.src0, p.src_ld0, p.sh0, p.sw0);
  if (p.nsrc > 1) src_add((const T*)p.src1, p.src_ld1, p.sh1, p.sw1);
  if (p.nsrc > 2) src_add((const T*)p.src2, p.src_ld2, p.sh2, p.sw2);
  auto finish = [&](int xx, float* v) {
    const long long pix = (long long)row * p.w + xx;
    T* yp = (T*)p.y + pix * p.y_ld + c;
    float t[VW];
    if (p.res) {
      VecN<T, VW>::load((const T*)p.res + pix * p.res_ld + c, t);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] += t[k];
    }
    if (p.beta) {
      VecN<T, VW>::load(yp, t);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] += t[k];
    }
    if (p.act) {
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      VecN<T, VW>::load((const T*)p.z + pix * p.z_ld + c, t);
#pragma unroll
      for (int k = 0; k < VW; ++k) v[k] *= act_dz(t[k], p.dact, p.alpha);
    }
    VecN<T, VW>::store(yp, v);
  };
  finish(x, v0);
  if (two) finish(x + 1, v1);
}

// EW_FUSE of ONE source upsampled by an integer ratio R (align_corners False; HRNet's fuse
// and concat upsamples, R = 2 / 4), bf16 x8: a thread owns the R output columns R q .. R q + R - 1
// of one output row, whose bilinear columns all lie in {q - 1, q, q + 1}: 2 rows x 3 column
// loads per R outputs (ew_fuse2_kernel: 6 per 2).  Per output the lerp indices, weights and
// arithmetic are up_sample_add's (lerp_src), so the results are the same as ew_kernel's.
template <int R>
__global__ __launch_bounds__(256) void ew_fuser_kernel(const dvie_ew_desc p, int cq) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int sw = p.sw0, sh = p.sh0;
  if (e >= sw * cq) return;
  const int q = e / cq;
  const int c = (e - q * cq) * 8;
  const int row = blockIdx.y;
  const int n = row / p.h, y = row - (row / p.h) * p.h;
  const bf16_t* s = (const bf16_t*)p.src0;
  const long long ld = p.src_ld0;
  const Lerp ly = lerp_src(y, sh, p.h, 0);
  const long long r0 = ((long long)n * sh + ly.i0) * sw, r1 = ((long long)n * sh + ly.i1) * sw;
  const int qm = q > 0 ? q - 1 : 0, qp = q + 1 < sw ? q + 1 : sw - 1;
  float tm0[8], t00[8], tp0[8], tm1[8], t01[8], tp1[8];
  VecN<bf16_t, 8>::load(s + (r0 + qm) * ld + c, tm0);
  VecN<bf16_t, 8>::load(s + (r0 + q) * ld + c, t00);
  VecN<bf16_t, 8>::load(s + (r0 + qp) * ld + c, tp0);
  VecN<bf16_t, 8>::load(s + (r1 + qm) * ld + c, tm1);
  VecN<bf16_t, 8>::load(s + (r1 + q) * ld + c, t01);
  VecN<bf16_t, 8>::load(s + (r1 + qp) * ld + c, tp1);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int x = R * q + r;
    if (x >= p.w) break;
    const Lerp lx = lerp_src(x, sw, p.w, 0);  // lx.i0 in {q - 1, q}, lx.i1 in {q, q + 1}
    const bool lo = lx.i0 < q, hi = lx.i1 > q;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = lo ? tm0[k] : t00[k], b = hi ? tp0[k] : t00[k];
      const float cc = lo ? tm1[k] : t01[k], d = hi ? tp1[k] : t01[k];
      v[k] = 0.f + (ly.l0 * (lx.l0 * a + lx.l1 * b) + ly.l1 * (lx.l0 * cc + lx.l1 * d));
    }
    const long long pix = (long long)row * p.w + x;
    bf16_t* yp = (bf16_t*)p.y + pix * p.y_ld + c;
    float t[8];
    if (p.res) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.res + pix * p.res_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.beta) {
      VecN<bf16_t, 8>::load(yp, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.act) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.z + pix * p.z_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= act_dz(t[k], p.dact, p.alpha);
    }
    VecN<bf16_t, 8>::store(yp, v);
  }
}

// EW_UPT (the upsample adjoint) at an integer ratio R (align_corners False), bf16 x8, with two
// horizontally adjacent coarse outputs per thread: their fine-column windows (2R + 2 each,
// R apart) overlap, so a fine row costs 3R + 2 loads per pair instead of 4R + 4.  Same
// weights (upt_weight) and, per output, the same summation order as upt_ratio.  Launched for
// R = 2 (8x128x256 128-ch: 0.142 -> 0.110 ms/step, 64-ch 0.129 -> 0.115, profiles/r05h/);
// at R = 4 it measured no gain (0.187 vs 0.190: 172 VGPRs, half the occupancy).
template <int R>
__global__ __launch_bounds__(256) void ew_upt2_kernel(const dvie_ew_desc p, int cq) {
  constexpr int NC = 2 * R + 2, NC2 = 3 * R + 2;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int wp = (p.w + 1) >> 1;
  if (e >= wp * cq) return;
  const int xp = e / cq;
  const int c = (e - xp * cq) * 8;
  const int x = 2 * xp;
  const bool two = x + 1 < p.w;
  const int row = blockIdx.y;
  const int n = row / p.h, y = row - (row / p.h) * p.h;
  const int sh = p.sh0, sw = p.sw0;
  const bf16_t* s = (const bf16_t*)p.src0;
  const long long ld = p.src_ld0;
  const int Y0 = R * y - R / 2 - 1, X0 = R * x - R / 2 - 1;
  // column j of the pair's window: fine X0 + j; pixel x uses j < NC, pixel x + 1 uses j >= R
  float wx0[NC2], wx1[NC2];
  unsigned xo[NC2];  // byte offset of the column's 8 channels within a fine row
#pragma unroll
  for (int j = 0; j < NC2; ++j) {
    const int X = X0 + j;
    const bool in = X >= 0 && X < sw;
    wx0[j] = (in && j < NC) ? upt_weight(X, x, p.w, sw, 0) : 0.f;
    wx1[j] = (in && two && j >= R) ? upt_weight(X, x + 1, p.w, sw, 0) : 0.f;
    xo[j] = (unsigned)((in ? X : 0) * ld + c) * 2u;
  }
  // (32-bit buffer offsets: the launch checks the source spans < 4 GB)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)s, 0, 0x7FFFFFF0, 0x00020000);
  float v0[8], v1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v0[k] = v1[k] = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int Y = Y0 + i;
    if (Y < 0 || Y >= sh) continue;
    const float wy = upt_weight(Y, y, p.h, sh, 0);
    if (wy == 0.f) continue;
    const unsigned rowo = (unsigned)(((long long)n * sh + Y) * sw * ld) * 2u;
    i32x4 raw[NC2];
#pragma unroll
    for (int j = 0; j < NC2; ++j) raw[j] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, rowo + xo[j], 0, 0));
#pragma unroll
    for (int j = 0; j < NC2; ++j) {
      const float g0 = wy * wx0[j], g1 = wy * wx1[j];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = __uint_as_float(((uint32_t)raw[j][k]) << 16), hi = __uint_as_float(((uint32_t)raw[j][k]) & 0xffff0000u);
        if (j < NC) {
          v0[2 * k] += g0 * lo;
          v0[2 * k + 1] += g0 * hi;
        }
        if (j >= R) {
          v1[2 * k] += g1 * lo;
          v1[2 * k + 1] += g1 * hi;
        }
      }
    }
  }
  auto finish = [&](int xx, float* v) {
    const long long pix = (long long)row * p.w + xx;
    bf16_t* yp = (bf16_t*)p.y + pix * p.y_ld + c;
    float t[8];
    if (p.res) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.res + pix * p.res_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.beta) {
      VecN<bf16_t, 8>::load(yp, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.act) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.z + pix * p.z_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= act_dz(t[k], p.dact, p.alpha);
    }
    VecN<bf16_t, 8>::store(yp, v);
  };
  finish(x, v0);
  if (two) finish(x + 1, v1);
}

// EW_UPT at an integer ratio R (align_corners False), bf16 x8, 2 x 2 coarse outputs per thread
// (coarse rows y, y + 1, columns x, x + 1): the fine pixels reaching coarse i are exactly
// R i - R/2 .. R i + R + R/2 - 1 per axis (the forward's lerp; edge clamping keeps them inside),
// so the four outputs read one 3R x 3R fine box: (3R)^2 / 4 loads per output (R = 4: 36, against
// 80 for upt_ratio's 2R + 2 candidates; R = 2: 9 against ew_upt2_kernel's 16).  Separable: each
// fine row is first combined across the columns (weights upt_weight, as the forward), then
// added into the rows' outputs with the row weights.  fp32 accumulation; the summation order
// differs from upt_ratio's (row partials first), so results agree to fp32 rounding.
template <int R>
__global__ __launch_bounds__(256) void ew_upt22_kernel(const dvie_ew_desc p, int cq) {
  constexpr int NW = 3 * R;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int wp = (p.w + 1) >> 1, hp = (p.h + 1) >> 1;
  if (e >= wp * cq) return;
  const int xp = e / cq;
  const int c = (e - xp * cq) * 8;
  const int x = 2 * xp;
  const int rowp = blockIdx.y;
  const int n = rowp / hp, y = 2 * (rowp - (rowp / hp) * hp);
  const bool twox = x + 1 < p.w, twoy = y + 1 < p.h;
  const int sh = p.sh0, sw = p.sw0;
  const long long ld = p.src_ld0;
  const int Y0 = R * y - R / 2, X0 = R * x - R / 2;
  float wx0[NW], wx1[NW];
  unsigned xo[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int X = X0 + j;
    const bool in = X >= 0 && X < sw;
    wx0[j] = in ? upt_weight(X, x, p.w, sw, 0) : 0.f;
    wx1[j] = (in && twox) ? upt_weight(X, x + 1, p.w, sw, 0) : 0.f;
    xo[j] = (unsigned)((in ? X : 0) * ld + c) * 2u;
  }
  // (32-bit buffer offsets: the launch checks the source span < 2 GB)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.src0, 0, 0x7FFFFFF0, 0x00020000);
  float acc[2][2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[a][b][k] = 0.f;
#pragma unroll 1
  for (int i = 0; i < NW; ++i) {
    const int Y = Y0 + i;
    if (Y < 0 || Y >= sh) continue;
    const float wy0 = upt_weight(Y, y, p.h, sh, 0), wy1 = twoy ? upt_weight(Y, y + 1, p.h, sh, 0) : 0.f;
    if (wy0 == 0.f && wy1 == 0.f) continue;
    const unsigned rowo = (unsigned)(((long long)n * sh + Y) * sw * ld) * 2u;
    i32x4 raw[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) raw[j] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, rowo + xo[j], 0, 0));
    float h0[8], h1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h0[k] = h1[k] = 0.f;
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = __uint_as_float(((uint32_t)raw[j][k]) << 16), hi = __uint_as_float(((uint32_t)raw[j][k]) & 0xffff0000u);
        h0[2 * k] += wx0[j] * lo;
        h0[2 * k + 1] += wx0[j] * hi;
        h1[2 * k] += wx1[j] * lo;
        h1[2 * k + 1] += wx1[j] * hi;
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      acc[0][0][k] += wy0 * h0[k];
      acc[0][1][k] += wy0 * h1[k];
      acc[1][0][k] += wy1 * h0[k];
      acc[1][1][k] += wy1 * h1[k];
    }
  }
  auto finish = [&](int yy, int xx, float* v) {
    const long long pix = ((long long)n * p.h + yy) * p.w + xx;
    bf16_t* yp = (bf16_t*)p.y + pix * p.y_ld + c;
    float t[8];
    if (p.res) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.res + pix * p.res_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.beta) {
      VecN<bf16_t, 8>::load(yp, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (p.act) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      VecN<bf16_t, 8>::load((const bf16_t*)p.z + pix * p.z_ld + c, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= act_dz(t[k], p.dact, p.alpha);
    }
    VecN<bf16_t, 8>::store(yp, v);
  };
  finish(y, x, acc[0][0]);
  if (twox) finish(y, x + 1, acc[0][1]);
  if (twoy) {
    finish(y + 1, x, acc[1][0]);
    if (twox) finish(y + 1, x + 1, acc[1][1]);
  }
}

// EW_NCHW for bf16 x8 without epilogue operands: one PIXEL per thread, consecutive threads on
// consecutive x, so every planar read (one channel of 64 pixels per wave) is a contiguous
// 256-B row piece -- the generic kernel's channel-fastest mapping made them 4-byte gathers
// H x W floats apart.  The thread then writes its pixel's c channels as 16-B vectors.
__global__ __launch_bounds__(256) void ew_nchw_kernel(const dvie_ew_desc p) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= p.w) return;
  const int row = blockIdx.y;
  const int n = row / p.h, y = row - (row / p.h) * p.h;
  const long long pix = (long long)row * p.w + x;
  const long long base = (long long)n * p.sn + (long long)y * p.sh + (long long)x * p.sw;
  if (p.c <= 32) {  // every planar load issued before the first store (the stores may alias)
    float v[32];
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) {
      float t = 0.f;
      if (ch < p.c && ch < p.ext_c) {
        const bool second = p.src1 != nullptr && ch >= p.sh1;
        const float* e = second ? (const float*)p.src1 : p.ext;
        const int cc = second ? ch - p.sh1 : ch;
        t = e[base + (long long)cc * p.sc];
        if (p.mean) t = (t - p.mean[ch]) / p.std[ch];
      }
      v[ch] = t;
    }
#pragma unroll
    for (int c = 0; c < 32; c += 8)
      if (c < p.c) VecN<bf16_t, 8>::store((bf16_t*)p.y + pix * p.y_ld + c, v + c);
    return;
  }
  for (int c = 0; c < p.c; c += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = c + k;
      float t = 0.f;
      if (ch < p.ext_c) {
        const bool second = p.src1 != nullptr && ch >= p.sh1;
        const float* e = second ? (const float*)p.src1 : p.ext;
        const int cc = second ? ch - p.sh1 : ch;
        t = e[base + (long long)cc * p.sc];
        if (p.mean) t = (t - p.mean[ch]) / p.std[ch];
      }
      v[k] = t;
    }
    VecN<bf16_t, 8>::store((bf16_t*)p.y + pix * p.y_ld + c, v);
  }
}

}  // namespace dvie

using namespace dvie;

// DVIE_EW_FUSE2=0: one output pixel per thread for the fuse op (A/B runs); read per launch
static bool fuse2_on() {
  const char* e = getenv("DVIE_EW_FUSE2");
  return !(e && *e == '0');
}

// DVIE_EW_FUSER: single-source integer-ratio fuse ops on ew_fuser_kernel -- 1 (default) at
// ratio 4, 2 at ratios 2 and 4, 0 never (A/B runs)
static int fuser_on() {
  const char* e = getenv("DVIE_EW_FUSER");
  return e && *e ? atoi(e) : 1;
}

// DVIE_EW_UPT22=0: the integer-ratio upsample adjoint without the 2 x 2-output kernel (A/B)
static bool upt22_on() {
  const char* e = getenv("DVIE_EW_UPT22");
  return !(e && *e == '0');
}

// DVIE_EW_UPT2=0: one coarse output per thread for the integer-ratio upsample adjoint (A/B)
static bool upt2_on() {
  const char* e = getenv("DVIE_EW_UPT2");
  return !(e && *e == '0');
}

extern "C" int dvie_ew(const dvie_ew_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->c > 0 && d->c % 4 == 0, "ew: c=%d must be a multiple of 4", d ? d->c : -1);
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0, "ew: empty shape");
  DVIE_CHECK_ARG(d->op == DVIE_EW_TONCHW || (d->y && d->y_ld % 4 == 0), "ew: y");
  if (d->op == DVIE_EW_POOL) DVIE_CHECK_ARG(d->sh0 == 2 * d->h && d->sw0 == 2 * d->w, "ew: pool shape");
  if (d->op == DVIE_EW_POOLT) DVIE_CHECK_ARG(d->h == 2 * d->sh0 && d->w == 2 * d->sw0, "ew: poolT shape");
  if (d->op == DVIE_EW_NCHW || d->op == DVIE_EW_TONCHW || d->op == DVIE_EW_MASK)
    DVIE_CHECK_ARG(d->ext != nullptr, "ew: ext");
  if (d->dact) DVIE_CHECK_ARG(d->z != nullptr && d->z_ld % 4 == 0, "ew: z");
  if (d->op == DVIE_EW_IM2COL)
    DVIE_CHECK_ARG(d->ext_c > 0 && d->ext_c % 8 == 0 && d->src0 && d->src_ld0 >= d->ext_c &&
                       d->sh0 > 0 && d->sw0 > 0 && d->sh0 * d->sw0 * d->ext_c <= d->c,
                   "ew: im2col ext_c=%d c=%d taps=%dx%d", d->ext_c, d->c, d->sh0, d->sw0);
  DVIE_CHECK_ARG((long long)d->n * d->h < 65536 && (long long)d->w * d->c < (1LL << 30), "ew: grid too large");
  hipStream_t s = (hipStream_t)stream;
  // 16-byte vectors for bf16 when every operand allows it
  auto al = [](const void* q, long long ld) { return !q || ((((uintptr_t)q) & 15) == 0 && ld % 8 == 0); };
  const bool v8 = d->dtype == DVIE_BF16 && d->c % 8 == 0 && al(d->y, d->y_ld) && al(d->src0, d->src_ld0) &&
                  al(d->src1, d->src_ld1) && al(d->src2, d->src_ld2) && al(d->res, d->res_ld) && al(d->z, d->z_ld);
  const int vw = v8 ? 8 : 4;
  const int cq = d->c / vw;
  const dim3 grid((unsigned)((d->w * cq + 255) / 256), (unsigned)(d->n * d->h));
  if (d->dtype == DVIE_BF16) {
    if (v8) {
      // (pairs need every source at most the output's size: a source step <= 1 per pixel)
      const bool up = d->sw0 <= d->w && d->sh0 <= d->h && (d->nsrc < 2 || (d->sw1 <= d->w && d->sh1 <= d->h)) &&
                      (d->nsrc < 3 || (d->sw2 <= d->w && d->sh2 <= d->h));
      if (d->op == DVIE_EW_NCHW && !d->res && !d->beta && !d->act && !d->dact) {
        const dim3 gn((unsigned)((d->w + 255) / 256), (unsigned)(d->n * d->h));
        DVIE_LAUNCH(ew_nchw_kernel, gn, dim3(256), 0, s, *d);
      } else if (d->op == DVIE_EW_FUSE && d->nsrc == 1 && !d->align && fuser_on() &&
                 ((d->h == 4 * d->sh0 && d->w == 4 * d->sw0) || (fuser_on() > 1 && d->h == 2 * d->sh0 && d->w == 2 * d->sw0))) {
        // ratio 4 only by default: the 4x 256-channel concat upsample 0.190 -> 0.167 ms/step, while
        // at ratio 2 the pair kernel measured faster (0.092 vs 0.097 ms, profiles/r06/ew_ab_*)
        const dim3 gr((unsigned)((d->sw0 * cq + 255) / 256), (unsigned)(d->n * d->h));
        if (d->w == 4 * d->sw0)
          DVIE_LAUNCH((ew_fuser_kernel<4>), gr, dim3(256), 0, s, *d, cq);
        else
          DVIE_LAUNCH((ew_fuser_kernel<2>), gr, dim3(256), 0, s, *d, cq);
      } else if (d->op == DVIE_EW_FUSE && up && fuse2_on()) {
        const dim3 g2((unsigned)((((d->w + 1) / 2) * cq + 255) / 256), (unsigned)(d->n * d->h));
        DVIE_LAUNCH((ew_fuse2_kernel<bf16_t, 8>), g2, dim3(256), 0, s, *d, cq);
      } else if (d->op == DVIE_EW_FUSE)
        DVIE_LAUNCH((ew_kernel<bf16_t, 8, DVIE_EW_FUSE>), grid, dim3(256), 0, s, *d, cq);
      else if (d->op == DVIE_EW_UPT && !d->align && upt22_on() &&
               (unsigned long long)d->n * d->sh0 * d->sw0 * d->src_ld0 * 2ull < 0x7FFFFFF0ull &&
               ((d->sh0 == 2 * d->h && d->sw0 == 2 * d->w) || (d->sh0 == 4 * d->h && d->sw0 == 4 * d->w))) {
        const dim3 g4((unsigned)((((d->w + 1) / 2) * cq + 255) / 256), (unsigned)(d->n * ((d->h + 1) / 2)));
        if (d->sh0 == 4 * d->h)
          DVIE_LAUNCH((ew_upt22_kernel<4>), g4, dim3(256), 0, s, *d, cq);
        else
          DVIE_LAUNCH((ew_upt22_kernel<2>), g4, dim3(256), 0, s, *d, cq);
      } else if (d->op == DVIE_EW_UPT && !d->align && upt2_on() &&
               (unsigned long long)d->n * d->sh0 * d->sw0 * d->src_ld0 * 2ull < 0x7FFFFFF0ull &&
               (d->sh0 == 2 * d->h && d->sw0 == 2 * d->w)) {
        const dim3 g2((unsigned)((((d->w + 1) / 2) * cq + 255) / 256), (unsigned)(d->n * d->h));
        DVIE_LAUNCH((ew_upt2_kernel<2>), g2, dim3(256), 0, s, *d, cq);
      } else if (d->op == DVIE_EW_UPT)
        DVIE_LAUNCH((ew_kernel<bf16_t, 8, DVIE_EW_UPT>), grid, dim3(256), 0, s, *d, cq);
      else
        DVIE_LAUNCH((ew_kernel<bf16_t, 8, -2>), grid, dim3(256), 0, s, *d, cq);
    } else {
      DVIE_LAUNCH((ew_kernel<bf16_t, 4, -1>), grid, dim3(256), 0, s, *d, cq);
    }
  } else {
    DVIE_LAUNCH((ew_kernel<float, 4, -1>), grid, dim3(256), 0, s, *d, cq);
  }
  DVIE_RETURN_LAUNCH();
}
