// Implicit-GEMM convolution for gfx950 (forward, and data-gradient as a forward conv over
// the output gradient with re-packed weights) — v2.
//
// GEMM: rows = output channels (MFMA "A" operand: packed weights [cout][kpad]),
// columns = output pixels (MFMA "B" operand: NHWC input gathered per tap), K = taps*c.
// Both operands are K-contiguous, so the LDS images are 128-byte rows (8 x 16-B chunks,
// XOR-swizzled by row) of either operand.
//
// * Staging: LDS-DMA (`buffer_load_dwordx4 ... lds`) straight from HBM/L2 into the
//   swizzled image — no VGPR staging, no ds_write.  The swizzle is applied to each lane's
//   SOURCE chunk (the DMA destination is lane-linear).  The buffer resource's range check
//   turns every out-of-image tap (conv zero padding) and every row past cout into zeros.
//   Two LDS buffers: K-step t+1 is in flight while the MFMAs of K-step t run; one
//   vmcnt(0)+barrier per K-step.
// * MFMA: bf16 v_mfma_f32_16x16x32_bf16 / fp32 v_mfma_f32_16x16x4_f32 (exact fp32 chain).
// * Epilogue through LDS: accumulators are written as an fp32 [pixel][channel] tile, then
//   every thread handles one 16-byte chunk of an output pixel row, so bias / residual /
//   accumulate / activation / activation-derivative operands are read and the result is
//   written with coalesced 16-byte accesses (whole channel rows per pixel).
// * Blocks are 1-D: id -> (co tile fastest, pixel tile), remapped so that each XCD gets a
//   contiguous range (the co tiles of a pixel tile and neighbouring pixel tiles, which
//   share input rows, hit the same L2).
//
// Reference ops replaced: nn.Conv2d forward / backward-data in nets/HRNet.py and
// nets/vgg.py (every conv on the hot path).
#include "common.h"

namespace dvie {

template <typename T>
__device__ __forceinline__ void mfma_chunk(f32x4& acc, const i32x4& a, const i32x4& b);

template <>
__device__ __forceinline__ void mfma_chunk<float>(f32x4& acc, const i32x4& a, const i32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[0]), __int_as_float(b[0]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[1]), __int_as_float(b[1]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[2]), __int_as_float(b[2]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[3]), __int_as_float(b[3]), acc, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mfma_chunk<bf16_t>(f32x4& acc, const i32x4& a, const i32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                acc, 0, 0, 0);
}

__device__ __forceinline__ int swz128(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 8 output elements (OutT) <-> floats, 16 bytes
template <typename OT>
struct Out16;
template <>
struct Out16<bf16_t> {
  static constexpr int N = 8;
  __device__ static void load(const bf16_t* p, float* v) {
    const i32x4 r = *(const i32x4*)p;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(((uint32_t)r[k]) << 16);
      v[2 * k + 1] = __uint_as_float(((uint32_t)r[k]) & 0xffff0000u);
    }
  }
  __device__ static void store(bf16_t* p, const float* v) {
    i32x4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = (int)((uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16));
    *(i32x4*)p = r;
  }
};
template <>
struct Out16<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float* v) {
    const f32x4 r = *(const f32x4*)p;
    v[0] = r[0];
    v[1] = r[1];
    v[2] = r[2];
    v[3] = r[3];
  }
  __device__ static void store(float* p, const float* v) { *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]}; }
};

template <typename T, int N>
__device__ __forceinline__ void load_n(const T* p, float* v) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      const f32x4 r = *(const f32x4*)(p + k);
      v[k] = r[0];
      v[k + 1] = r[1];
      v[k + 2] = r[2];
      v[k + 3] = r[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      const f32x4 r = V4<bf16_t>::load(p + k);
      v[k] = r[0];
      v[k + 1] = r[1];
      v[k + 2] = r[2];
      v[k + 3] = r[3];
    }
  }
}

__device__ __forceinline__ int xcd_remap(int b, int nb) {
  // blocks b and b+8 share an XCD under round-robin dispatch: give XCD-group g the
  // contiguous range of logical ids [start_g, start_g + len_g)  (bijective for any nb)
  const int g = b & 7, i = b >> 3;
  const int q = nb >> 3, r = nb & 7;
  const int start = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
  return start + i;
}

template <typename T, int BC, int BP, int WC, int WP, bool OUTF32>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const dvie_conv_desc p, int n_ct, int n_tiles) {
  typedef typename std::conditional<OUTF32, float, T>::type OutT;
  constexpr int ES = sizeof(T);
  constexpr int VEC = 16 / ES;
  constexpr int KSTEP = 128 / ES;
  constexpr int TM = BC / WC / 16;
  constexpr int TN = BP / WP / 16;
  constexpr int AQ = BC / 32;  // LDS-DMA instructions per wave per stage (A), 8 rows each
  constexpr int BQ = BP / 32;
  constexpr int STAGE = (BC + BP) * 128;
  constexpr int EROW = BC * 4 + 16;
  constexpr int SMEM = (2 * STAGE > BP * EROW) ? 2 * STAGE : BP * EROW;
  static_assert(WC * WP == 4, "4 waves");
  static_assert(BC % 32 == 0 && BP % 32 == 0, "tiles of 32");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / WP, wp = wave % WP;
  const int bid = xcd_remap(blockIdx.x, n_tiles);
  const int c0 = (bid % n_ct) * BC;
  const long long p0 = (long long)(bid / n_ct) * BP;
  const int hw = p.oh * p.ow;
  const long long npix = (long long)p.n * hw;
  const int ntap = p.th * p.tw;
  const int K = ntap * p.c;
  const int CV = p.c / VEC;
  const int nk = (K + KSTEP - 1) / KSTEP;

  // buffer resources (wave-uniform): out-of-range offsets read as zero
  const unsigned long long wbytes = (unsigned long long)p.cout * p.kpad * ES;
  const unsigned long long xbytes = ((unsigned long long)p.n * p.ih * p.iw - 1) * p.x_ld * ES + (unsigned long long)p.c * ES;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)(wbytes < 0xFFFFFF00ull ? wbytes : 0xFFFFFF00ull), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)(xbytes < 0xFFFFFF00ull ? xbytes : 0xFFFFFF00ull), 0x00020000);
  constexpr unsigned OOB = 0xFFFFFFF0u;

  // per-lane A rows (weights) and B rows (pixels) this lane stages
  const int lr = lane >> 3;   // row within an 8-row DMA piece
  const int slot = lane & 7;  // 16-byte slot in the 128-byte LDS row
  unsigned a_off[AQ];
  int a_ch[AQ];
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    const int row = 8 * (wave + 4 * i) + lr;
    a_ch[i] = slot ^ ((row >> 1) & 7);
    a_off[i] = (unsigned)(((unsigned long long)(c0 + row) * p.kpad + a_ch[i] * VEC) * ES);
  }
  int bn[BQ], by[BQ], bx[BQ], b_ch[BQ];
#pragma unroll
  for (int i = 0; i < BQ; ++i) {
    const int row = 8 * (wave + 4 * i) + lr;
    b_ch[i] = slot ^ ((row >> 1) & 7);
    const long long pix = p0 + row;
    if (pix < npix) {
      const int n = (int)(pix / hw);
      const int r = (int)(pix - (long long)n * hw);
      const int oy = r / p.ow;
      bn[i] = n;
      by[i] = oy * p.sy;
      bx[i] = (r - oy * p.ow) * p.sx;
    } else {
      bn[i] = 0;
      by[i] = -(1 << 28);
      bx[i] = 0;
    }
  }

  auto stage = [&](int kt, int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BC * 128;
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      // (kept as a separate statement: with the offset expression inline, hipcc's host
      // pass silently drops the kernel's launch stub)
      const unsigned off = a_off[i] + (unsigned)(kt * KSTEP * ES);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(As + (wave + 4 * i) * 1024), 16, off, 0, 0, 0);
    }
    // K-step kt covers 16-byte vectors kv = 8*kt .. 8*kt+7, vector kv = (tap, cv)
    const int kv0 = kt * 8;
    const int t0 = kv0 / CV, cv0 = kv0 - t0 * CV;  // wave-uniform
    const int ti0 = t0 / p.tw, tj0 = t0 - ti0 * p.tw;
    const int t1 = t0 + 1, ti1 = t1 / p.tw, tj1 = t1 - ti1 * p.tw;
    const int dy0 = p.dy0 + ti0 * p.ddy, dx0 = p.dx0 + tj0 * p.ddx;
    const int dy1 = p.dy0 + ti1 * p.ddy, dx1 = p.dx0 + tj1 * p.ddx;
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      int tap, cv, dy, dx;
      if (CV >= 8) {  // uniform branch: a K-step spans at most two taps
        const int c = cv0 + b_ch[i];
        const bool wrap = c >= CV;
        tap = wrap ? t1 : t0;
        cv = wrap ? c - CV : c;
        dy = wrap ? dy1 : dy0;
        dx = wrap ? dx1 : dx0;
      } else {  // narrow inputs (c < 8 vectors): general decomposition
        const int kv = kv0 + b_ch[i];
        tap = kv / CV;
        cv = kv - tap * CV;
        const int ti = tap / p.tw;
        dy = p.dy0 + ti * p.ddy;
        dx = p.dx0 + (tap - ti * p.tw) * p.ddx;
      }
      const int iy = by[i] + dy, ix = bx[i] + dx;
      unsigned off = OOB;
      if (tap < ntap && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw)
        off = (unsigned)(((((unsigned long long)bn[i] * p.ih + iy) * p.iw + ix) * p.x_ld + (unsigned)cv * VEC) * ES);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(Bs + (wave + 4 * i) * 1024), 16, off, 0, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();

  const int r16 = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* As = smem + cur * STAGE;
    const char* Bs = As + BC * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + (lane >> 4);
      i32x4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const i32x4*)(As + swz128(wc * (BC / WC) + 16 * i + r16, ch));
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *(const i32x4*)(Bs + swz128(wp * (BP / WP) + 16 * j + r16, ch));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_chunk<T>(acc[i][j], af[i], bfr[j]);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS [pixel][channel] fp32 -> coalesced row chunks ----
  float* E = (float*)smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co_l = wc * (BC / WC) + 16 * i + 4 * (lane >> 4);
      const int px_l = wp * (BP / WP) + 16 * j + r16;
      *(f32x4*)((char*)E + px_l * EROW + co_l * 4) = acc[i][j];
    }
  __syncthreads();
  constexpr int OV = Out16<OutT>::N;
  constexpr int CPR = BC / OV;
  OutT* __restrict__ yg = (OutT*)p.y;
  const OutT* __restrict__ rg = (const OutT*)p.res;
  const T* __restrict__ zg = (const T*)p.z;
  for (int idx = tid; idx < BP * CPR; idx += 256) {
    const int px_l = idx / CPR;
    const int ck = idx - px_l * CPR;
    const int co = c0 + ck * OV;
    const long long pix = p0 + px_l;
    if (pix >= npix || co >= p.cout) continue;
    float v[OV];
    const char* er = (const char*)E + px_l * EROW + ck * OV * 4;
#pragma unroll
    for (int k = 0; k < OV; k += 4) {
      const f32x4 t = *(const f32x4*)(er + k * 4);
      v[k] = t[0];
      v[k + 1] = t[1];
      v[k + 2] = t[2];
      v[k + 3] = t[3];
    }
    const int n = (int)(pix / hw);
    const int r = (int)(pix - (long long)n * hw);
    const int oy = r / p.ow;
    const int ox = r - oy * p.ow;
    const long long yrow = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
    if (p.bias) {
#pragma unroll
      for (int k = 0; k < OV; k += 4) {
        const f32x4 b = *(const f32x4*)(p.bias + co + k);
        v[k] += b[0];
        v[k + 1] += b[1];
        v[k + 2] += b[2];
        v[k + 3] += b[3];
      }
    }
    if (rg) {
      float t[OV];
      Out16<OutT>::load(rg + yrow * p.res_ld + co, t);
#pragma unroll
      for (int k = 0; k < OV; ++k) v[k] += t[k];
    }
    if (p.beta) {
      float t[OV];
      Out16<OutT>::load(yg + yrow * p.y_ld + co, t);
#pragma unroll
      for (int k = 0; k < OV; ++k) v[k] += t[k];
    }
    if (p.act) {
#pragma unroll
      for (int k = 0; k < OV; ++k) v[k] = act_fwd(v[k], p.act, p.alpha);
    }
    if (p.dact) {
      float z[OV];
      load_n<T, OV>(zg + yrow * p.z_ld + co, z);
#pragma unroll
      for (int k = 0; k < OV; ++k) v[k] *= act_dz(z[k], p.dact, p.alpha);
    }
    Out16<OutT>::store(yg + yrow * p.y_ld + co, v);
  }
}

template <typename T, int BC, int BP, int WC, int WP>
static void launch_conv(const dvie_conv_desc& p, hipStream_t s) {
  const long long npix = (long long)p.n * p.oh * p.ow;
  const int n_ct = (p.cout + BC - 1) / BC;
  const int n_tiles = (int)((npix + BP - 1) / BP) * n_ct;
  if (p.out_f32)
    DVIE_LAUNCH((conv_igemm_kernel<T, BC, BP, WC, WP, true>), dim3(n_tiles), dim3(256), 0, s, p, n_ct, n_tiles);
  else
    DVIE_LAUNCH((conv_igemm_kernel<T, BC, BP, WC, WP, false>), dim3(n_tiles), dim3(256), 0, s, p, n_ct,
                       n_tiles);
}

template <typename T>
static void dispatch_conv(const dvie_conv_desc& p, hipStream_t s) {
  const long long npix = (long long)p.n * p.oh * p.ow;
  const bool small = npix < 64LL * 512;  // too few 128-pixel tiles to fill 256 CUs
  if (p.cout <= 32) {
    if (small) launch_conv<T, 32, 64, 2, 2>(p, s);
    else launch_conv<T, 32, 128, 2, 2>(p, s);
  } else if (p.cout <= 64) {
    if (small) launch_conv<T, 64, 64, 2, 2>(p, s);
    else launch_conv<T, 64, 128, 2, 2>(p, s);
  } else {
    if (small) launch_conv<T, 128, 64, 2, 2>(p, s);
    else launch_conv<T, 128, 128, 2, 2>(p, s);
  }
}

bool conv_halo_launch(const dvie_conv_desc& p, hipStream_t s);  // conv_halo.hip
bool conv_halo_ph4_launch(const dvie_conv_desc& p, hipStream_t s);  // conv_halo.hip
bool conv1x1_launch(const dvie_conv_desc& p, hipStream_t s);    // conv1x1.hip
bool conv_s2_launch(const dvie_conv_desc& p, hipStream_t s);    // conv_s2.hip

}  // namespace dvie

using namespace dvie;

extern "C" int dvie_conv2d_fwd(const dvie_conv_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->x && d->w && d->y, "conv: null pointer");
  const int vec = d->dtype == DVIE_BF16 ? 8 : 4;
  const int es = d->dtype == DVIE_BF16 ? 2 : 4;
  const int ovec = (d->out_f32 || d->dtype == DVIE_F32) ? 4 : 8;
  DVIE_CHECK_ARG(d->c > 0 && d->c % vec == 0, "conv: c=%d must be a multiple of %d", d->c, vec);
  DVIE_CHECK_ARG(d->cout > 0 && d->cout % ovec == 0, "conv: cout=%d must be a multiple of %d", d->cout, ovec);
  DVIE_CHECK_ARG(d->kpad % 64 == 0 && d->kpad >= d->th * d->tw * d->c, "conv: kpad=%d", d->kpad);
  DVIE_CHECK_ARG(d->x_ld % vec == 0 && d->y_ld % ovec == 0 && (!d->res || d->res_ld % ovec == 0) &&
                     (!d->z || d->z_ld % ovec == 0),
                 "conv: ld alignment x_ld=%lld y_ld=%lld", d->x_ld, d->y_ld);
  DVIE_CHECK_ARG(d->th >= 1 && d->tw >= 1 && d->th * d->tw <= 64, "conv: taps");
  DVIE_CHECK_ARG(d->n > 0 && d->oh > 0 && d->ow > 0 && d->ih > 0 && d->iw > 0, "conv: empty shape");
  DVIE_CHECK_ARG(((uintptr_t)d->x & 15) == 0 && ((uintptr_t)d->w & 15) == 0 && ((uintptr_t)d->y & 15) == 0,
                 "conv: x/w/y not 16B aligned");
  DVIE_CHECK_ARG(!d->bias || ((uintptr_t)d->bias & 15) == 0, "conv: bias not 16B aligned");
  DVIE_CHECK_ARG(d->dtype == DVIE_BF16 || d->out_f32 || d->dtype == DVIE_F32, "conv: dtype");
  // The kernels address the input (and weights) through buffer resources with 32-bit
  // offsets.  A larger input is run as batch chunks whose input span fits: the images of
  // a batch are independent, so each chunk is the same conv over n' images with x / y /
  // res / z advanced by n0 images (the output keeps its own geometry yh x yw).
  const unsigned long long img_x = (unsigned long long)d->ih * d->iw * d->x_ld * es;
  const unsigned long long wb = (unsigned long long)d->cout * d->kpad * es;
  DVIE_CHECK_ARG(wb < 0xFFFFFF00ull, "conv: weights exceed the 4 GiB buffer range");
  DVIE_CHECK_ARG(img_x < 0xFFFFFF00ull, "conv: one input image exceeds the 4 GiB buffer range");
  hipStream_t s = (hipStream_t)stream;
  const long long chunk = (long long)(0xFFFFFF00ull / img_x) < d->n ? (long long)(0xFFFFFF00ull / img_x) : d->n;
  const int oes = (d->out_f32 || d->dtype == DVIE_F32) ? 4 : 2;
  const unsigned long long img_y = (unsigned long long)d->yh * d->yw;
  for (long long n0 = 0; n0 < d->n; n0 += chunk) {
    dvie_conv_desc c = *d;
    c.n = (int)(d->n - n0 < chunk ? d->n - n0 : chunk);
    c.x = (const char*)d->x + n0 * img_x;
    c.y = (char*)d->y + n0 * img_y * d->y_ld * oes;
    if (d->res) c.res = (const char*)d->res + n0 * img_y * d->res_ld * oes;
    if (d->z) c.z = (const char*)d->z + n0 * img_y * d->z_ld * es;
    if (c.phc) {  // the one-launch stride-2 data gradient: the halo kernel only
      DVIE_CHECK_ARG(conv_halo_ph4_launch(c, s), "conv: phase-split output (phc=%d) needs bf16, 2x2 taps at "
                     "(0,0), osy=osx=2, cout=4*phc, phc %% 32 == 0, no bias", c.phc);
      continue;
    }
    if (conv1x1_launch(c, s)) continue;
    if (conv_halo_launch(c, s)) continue;
    if (conv_s2_launch(c, s)) continue;
    if (c.dtype == DVIE_BF16)
      dispatch_conv<bf16_t>(c, s);
    else
      dispatch_conv<float>(c, s);
  }
  DVIE_RETURN_LAUNCH();
}
