// Halo-tile implicit-GEMM convolution for gfx950, bf16 (v3): stride-1 convolutions with a
// 1x1 or 3x3 tap grid whose output placement is the identity — every 3x3/1x1 forward conv
// of HRNet/VGG and the data gradient of the stride-1 ones (a 3x3 conv over the output
// gradient with flipped weights).
//
// Why a halo tile: the per-tap implicit GEMM (conv_fwd.hip) gathers every input pixel
// once per tap, i.e. 9x for a 3x3 conv, from L2 into LDS.  Here a workgroup owns PR
// output rows x 64 output columns; it stages the input halo of that tile, (PR+TH-1) x
// (64+TW-1) pixels x 64 channels, ONCE per 64-channel chunk and every tap reads its B
// fragments from that image at a row/column shift.  Only the weights are streamed per
// tap (BC rows x 128 B).
//
// * LDS images use a 144-byte row pitch (8 data slots + 1 pad slot of 16 B): the 16-lane
//   groups of ds_read_b128 then hit 16 distinct slots for any 16 distinct rows mod 16, so
//   the tap-shifted reads are conflict-free and every fragment address is the lane's base
//   plus a compile-time immediate (no per-tap address arithmetic).
// * Staging is LDS-DMA (buffer_load_dwordx4 ... lds): 64 lanes fill 64 consecutive slots;
//   each lane's source offset is precomputed once per workgroup.  Pad slots and taps that
//   fall outside the image carry an out-of-range offset and land as zeros (conv padding).
//   The chunk offset is folded into the buffer resource's base, so the precomputed
//   offsets stay valid for every chunk.
// * Pipeline: one step = (chunk, tap).  Step s+1's weight tile and a 1/NT share of the
//   NEXT chunk's halo are issued before the MFMAs of step s; one vmcnt(0)+barrier per step.
// * MFMA v_mfma_f32_32x32x16_bf16; a wave owns 32*TM output channels x TNR output rows of
//   64 pixels.  Epilogue through LDS as in conv_fwd.hip (coalesced 16-B row chunks, fused
//   bias / residual / accumulate / activation / activation-derivative).
//
// Reference ops replaced: nn.Conv2d forward / backward-data (nets/HRNet.py, nets/vgg.py).
#include <stdlib.h>
#include <string.h>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

__device__ __forceinline__ int xcd_remap3(int b, int nb) {
  const int g = b & 7, i = b >> 3;
  const int q = nb >> 3, r = nb & 7;
  const int start = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
  return start + i;
}

// F32OUT: the epilogue stores fp32 (e.g. the fp32 head outputs of a bf16 plan): ELU / tanh
// through expm1f / tanhf; the short v_exp_f32 forms (common.h) are for bf16 stores only
template <bool F32OUT = false>
__device__ __forceinline__ void act_apply(float* v, int n, int act, float alpha) {
  if (act == DVIE_ACT_LRELU) {
    for (int k = 0; k < n; ++k) v[k] = v[k] > 0.f ? v[k] : v[k] * alpha;
  } else if (act == DVIE_ACT_RELU) {
    for (int k = 0; k < n; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
  } else if (act == DVIE_ACT_ELU) {
    for (int k = 0; k < n; ++k) v[k] = F32OUT ? (v[k] > 0.f ? v[k] : expm1f(v[k])) : elu_bf(v[k]);
  } else if (act == DVIE_ACT_TANH) {
    for (int k = 0; k < n; ++k) v[k] = F32OUT ? tanhf(v[k]) : tanh_bf(v[k]);
  }
}

__device__ __forceinline__ void dact_apply(float* v, const float* z, int n, int dact, float alpha) {
  if (dact == DVIE_ACT_LRELU) {
    for (int k = 0; k < n; ++k) v[k] *= z[k] > 0.f ? 1.f : alpha;
  } else if (dact == DVIE_ACT_RELU) {
    for (int k = 0; k < n; ++k) v[k] = z[k] > 0.f ? v[k] : 0.f;
  } else if (dact == DVIE_ACT_ELU) {
    for (int k = 0; k < n; ++k) v[k] *= z[k] > 0.f ? 1.f : z[k] + 1.f;
  } else if (dact == DVIE_ACT_TANH) {
    for (int k = 0; k < n; ++k) v[k] *= 1.f - z[k] * z[k];
  }
}

template <int TM, int WC, int WP, int TH, int TW>
struct HaloCfg {
  static constexpr int NW = WC * WP;               // waves per workgroup
  static constexpr int NTH = NW * 64;
  static constexpr int BC = 32 * TM * WC;          // output channels per tile
  static constexpr int PR = WP;                    // output rows per tile (one per row-wave)
  static constexpr int NT = TH * TW;               // taps
  static constexpr int HR = PR + TH - 1;           // halo rows
  static constexpr int HWD = 64 + TW - 1;          // halo columns
  static constexpr int PITCH = 144;                // bytes per LDS row (8 data + 1 pad slot)
  static constexpr int HSLOTS = HR * HWD * 9;
  static constexpr int NHI = ((HSLOTS + 63) / 64 + NW - 1) / NW * NW;  // DMA pieces per halo image
  static constexpr int NHQ = NHI / NW;             // pieces per wave (exact)
  static constexpr int HSZ = NHI * 1024;
  static constexpr int NH = NT > 1 ? 2 : 3;        // halo buffers
  // weight tile: BC rows x 128 B, XOR-swizzled 16-B chunks (rows are read at fixed offsets,
  // so the swizzle costs no per-step address arithmetic); BC/8 DMA pieces
  static constexpr int NAI = BC / 8;
  static constexpr int NAQ = (NAI + NW - 1) / NW;  // pieces per wave (upper bound)
  static constexpr int ASZ = BC * 128;
  static constexpr int NA = 3;                     // weight buffers (two steps of look-ahead)
  static constexpr int SMEM = NH * HSZ + NA * ASZ;
  // NT > 1: the next job's halo is issued in shares during taps 0..NT-2 of the current job
  static constexpr int SPREAD = NT > 1 ? NT - 1 : 1;
  __host__ __device__ static constexpr int q0(int t) { return t >= SPREAD ? NHQ : t * NHQ / SPREAD; }
  __host__ __device__ static constexpr int q1(int t) { return t >= SPREAD ? NHQ : (t + 1) * NHQ / SPREAD; }
};

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt left at their maxima)
#define DVIE_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4) | (15 << 8))
// vmcnt(n) and lgkmcnt(0) together
#define DVIE_VMCNT_LGKM0(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4))
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define DVIE_VMCASE(N) \
  case N:              \
    DVIE_VMCNT(N);     \
    break;
    DVIE_VMCASE(0) DVIE_VMCASE(1) DVIE_VMCASE(2) DVIE_VMCASE(3) DVIE_VMCASE(4) DVIE_VMCASE(5) DVIE_VMCASE(6)
    DVIE_VMCASE(7) DVIE_VMCASE(8) DVIE_VMCASE(9) DVIE_VMCASE(10) DVIE_VMCASE(11) DVIE_VMCASE(12) DVIE_VMCASE(13)
    DVIE_VMCASE(14) DVIE_VMCASE(15) DVIE_VMCASE(16) DVIE_VMCASE(17) DVIE_VMCASE(18) DVIE_VMCASE(19) DVIE_VMCASE(20)
    DVIE_VMCASE(21) DVIE_VMCASE(22) DVIE_VMCASE(23) DVIE_VMCASE(24) DVIE_VMCASE(25) DVIE_VMCASE(26) DVIE_VMCASE(27)
    DVIE_VMCASE(28) DVIE_VMCASE(29) DVIE_VMCASE(30) DVIE_VMCASE(31) DVIE_VMCASE(32) DVIE_VMCASE(33) DVIE_VMCASE(34)
    DVIE_VMCASE(35) DVIE_VMCASE(36) DVIE_VMCASE(37) DVIE_VMCASE(38) DVIE_VMCASE(39) DVIE_VMCASE(40) DVIE_VMCASE(41)
    DVIE_VMCASE(42) DVIE_VMCASE(43) DVIE_VMCASE(44) DVIE_VMCASE(45) DVIE_VMCASE(46) DVIE_VMCASE(47) DVIE_VMCASE(48)
#undef DVIE_VMCASE
    default: DVIE_VMCNT(0); break;
  }
}

struct JobInfo {
  int valid, t, k, c0, n, y0, x0;
};

// PH4 (TH = TW = 2, include/dvie.h dvie_conv_desc.phc): the stride-2 data gradient's four
// output phases in one launch.  Output channel block q of phc channels is phase (a, b) =
// ph4_a/b(q); it is placed at (2 oy + a, 2 ox + b) and uses tap (i, j) only if (i == 0 || a)
// and (j == 0 || b), so an accumulator block skips the MFMAs of the taps its phase lacks
// (9 of the 16 tap-phase products are nonzero).
__host__ __device__ constexpr int ph4_a(int q) { return q == 1 || q == 3; }
__host__ __device__ constexpr int ph4_b(int q) { return q == 1 || q == 2; }

template <int TM, int WC, int WP, int TH, int TW, bool OUTF32, bool PH4 = false>
__global__ __launch_bounds__(WC* WP * 64) void conv_halo_kernel(const dvie_conv_desc p, int n_ct, int n_tiles,
                                                                 int tiles_x, int tiles_y, int persistent,
                                                                 int epi_pre) {
  typedef HaloCfg<TM, WC, WP, TH, TW> C;
  static_assert(!PH4 || (TH == 2 && TW == 2 && !OUTF32), "phase-split output: 2 x 2 taps, bf16");
  constexpr int NW = C::NW;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / WP, wp = wave % WP;
  const int r32 = lane & 31, hh = lane >> 5;
  const int nchunks = (p.c + 63) >> 6;  // c < 64: one zero-padded chunk
  // epi_pre bit 1: static priority for the second-dispatched half of the waves (DVIE_SETPRIO)
  if ((epi_pre & 2) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const unsigned OOB = 0xFFFFFFF0u;

  // ---- tiles of this workgroup: one (remapped) tile, or an XCD-local strided range ----
  int tile0, tile_end, tile_step;
  if (!persistent) {
    tile0 = xcd_remap3(blockIdx.x, n_tiles);
    tile_end = tile0 + 1;
    tile_step = 1;
  } else {
    const int G = gridDim.x, g = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int nbg = G / 8 + (g < G % 8 ? 1 : 0);
    const int q = n_tiles / 8, r = n_tiles % 8;
    const int ts = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
    tile0 = ts + j;
    tile_end = ts + q + (g < r ? 1 : 0);
    tile_step = nbg;
  }
  if (tile0 >= tile_end) return;

  // jobs of this workgroup: (tile, chunk) in order; the tile is decoded only when it changes
  auto tile_job = [&](int t) {
    JobInfo J;
    J.t = t;
    J.k = 0;
    J.valid = t < tile_end;
    J.c0 = (t % n_ct) * C::BC;
    int pt = t / n_ct;
    J.x0 = (pt % tiles_x) * 64;
    pt /= tiles_x;
    J.y0 = (pt % tiles_y) * C::PR;
    J.n = pt / tiles_y;
    return J;
  };
  auto next_job = [&](const JobInfo& J) {
    if (J.k + 1 < nchunks) {
      JobInfo N = J;
      N.k = J.k + 1;
      return N;
    }
    return tile_job(J.t + tile_step);
  };

  // ---- per-lane DMA geometry (tile independent) ----
  int hgeo[C::NHQ];
#pragma unroll
  for (int q = 0; q < C::NHQ; ++q) {
    const int slot = (wave + NW * q) * 64 + lane;
    const int hr = slot / 9, cs = slot - 9 * (slot / 9);
    const int hy = hr / C::HWD, hx = hr - (hr / C::HWD) * C::HWD;
    hgeo[q] = (cs < 8 && cs * 8 < p.c && hr < C::HR * C::HWD) ? (hy << 16) | (hx << 4) | cs : -1;
  }
  // weight DMA: lane fills chunk (lane & 7) of row 8*piece + (lane >> 3) with source chunk
  // (lane & 7) ^ swz(row)
  unsigned aoff[C::NAQ];
#pragma unroll
  for (int q = 0; q < C::NAQ; ++q) {
    const int row = (wave + NW * q) * 8 + (lane >> 3);
    const int cs = (lane & 7) ^ ((row >> 1) & 7);
    aoff[q] = cs * 8 < p.c ? (unsigned)row * (unsigned)p.kpad * 2u + cs * 16u : OOB;
  }
  static_assert(C::NAI % NW == 0, "every wave issues the same number of weight pieces");
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;

  char* const Hs = smem;
  char* const As = smem + C::NH * C::HSZ;

  // halo pieces [qa, qb) of job J into halo buffer hb
  // (a job past the end still issues its pieces, with an empty buffer range: they land as
  // zeros in a buffer nobody reads, and every wave's vmcnt bookkeeping stays compile-time)
  auto halo_issue = [&](const JobInfo& J, int hb, int qa, int qb) {
    if (epi_pre & 16) return;  // timing experiments only (DVIE_HALO_DBG): no halo streaming
    const int nrec = J.valid ? (int)(xbytes - (unsigned long long)J.k * 128) : 0;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + (size_t)J.k * 128), 0, nrec, 0x00020000);
    char* dst = Hs + hb * C::HSZ + wave * 1024;
    const int ybase = J.y0 + p.dy0, xbase = J.x0 + p.dx0;
#pragma unroll
    for (int q = qa; q < qb; ++q) {
      const int gq = hgeo[q];
      const int iy = ybase + (gq >> 16), ix = xbase + ((gq >> 4) & 0xFFF);
      const bool ok = gq >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
      // (offset kept as a separate statement: with it inline, hipcc's host pass drops the
      // kernel's launch stub)
      const unsigned o = ok ? (unsigned)((J.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(gq & 15) * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(dst + q * NW * 1024), 16, o, 0, 0, 0);
    }
  };
  // weights of (job J, tap t) into weight buffer ab
  auto a_issue = [&](const JobInfo& J, int t, int ab) {
    if (epi_pre & 8) return;  // timing experiments only (DVIE_HALO_DBG): no weight streaming
    const unsigned o = (unsigned)((long long)J.c0 * p.kpad + t * p.c + 64 * J.k) * 2u;
    const int nrec = J.valid ? (int)((unsigned)p.cout * (unsigned)p.kpad * 2u - o) : 0;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.w + o), 0, nrec, 0x00020000);
    char* dst = As + ab * C::ASZ + wave * 1024;
#pragma unroll
    for (int q = 0; q < C::NAQ; ++q) {
      const unsigned ao = aoff[q];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(dst + q * NW * 1024), 16, ao, 0, 0, 0);
    }
  };

  f32x16 acc[TM][2];
  // A fragment addresses for the 4 k-slices (row r32 of the wave's 32-row blocks, chunk 2s+h)
  int a_off[4];
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    const int row = wc * 32 * TM + r32;
    a_off[sl] = row * 128 + (((2 * sl + hh) ^ ((row >> 1) & 7)) << 4);
  }
  const int b_base = (wp * C::HWD + r32) * C::PITCH + hh * 16;

  // ---- epilogue operands (bf16 output): residual, accumulate target and activation input
  // of the tile are loaded into registers during its last chunk, PRE_T steps before the
  // epilogue, so their HBM latency overlaps the remaining MFMAs instead of following them.
  // Buffer loads from a per-tile base: every wave issues the same count (lanes outside the
  // output get an out-of-range offset and load zeros), so the step's vmcnt stays exact.
  constexpr int PRE_T = C::NT >= 2 ? C::NT - 2 : 0;
  const bool PRE = !OUTF32 && (epi_pre & 1);
  const int npre = PRE ? TM * 4 * ((p.res ? 1 : 0) + (p.beta ? 1 : 0) + (p.dact ? 1 : 0)) : 0;
  i32x4 pre_r[TM][2][2], pre_b[TM][2][2], pre_z[TM][2][2];
  auto epi_prefetch = [&](const JobInfo& Jt) {
    const long long pix0 = ((long long)Jt.n * p.yh + (long long)Jt.y0 * p.osy + p.ory) * p.yw + (long long)Jt.x0 * p.osx + p.orx;
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16_t*)p.res + (p.res ? pix0 * p.res_ld : 0)), 0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16_t*)p.y + pix0 * p.y_ld), 0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16_t*)p.z + (p.dact ? pix0 * p.z_ld : 0)), 0, 0x7FFFFFF0, 0x00020000);
    const int oy = Jt.y0 + wp;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          const int ox = Jt.x0 + 32 * b + r32;
          int co = Jt.c0 + wc * 32 * TM + 32 * i + 16 * P + 8 * hh;
          bool ok = oy < p.oh && ox < p.ow && co < p.cout;
          long long dp = (long long)wp * p.osy * p.yw + (long long)(32 * b + r32) * p.osx;
          if constexpr (PH4) {  // phase (a, pb) of this block: placement offset, channel within the phase
            const int q = (Jt.c0 + wc * 32 * TM + 32 * i) / p.phc, a = ph4_a(q), pb = ph4_b(q);
            dp += (long long)a * p.yw + pb;
            co -= q * p.phc;
            ok = ok && 2 * oy + a < p.yh && 2 * ox + pb < p.yw;
          }
          const unsigned OFF = 0xFFFFFFF0u;
          if (p.res)
            pre_r[i][b][P] = __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? (unsigned)((dp * p.res_ld + co) * 2) : OFF, 0, 0);
          if (p.beta)
            pre_b[i][b][P] = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? (unsigned)((dp * p.y_ld + co) * 2) : OFF, 0, 0);
          if (p.dact)
            pre_z[i][b][P] = __builtin_amdgcn_raw_buffer_load_b128(rz, ok ? (unsigned)((dp * p.z_ld + co) * 2) : OFF, 0, 0);
        }
  };

  // ---- prologue: job 0 halo (+ job 1 for 1x1), weights of steps 0 and 1 ----
  const int dbg = DVIE_DBG(epi_pre & 24);
  epi_pre &= ~24;
  {
    const JobInfo J0 = tile_job(tile0);
    halo_issue(J0, 0, 0, C::NHQ);
    a_issue(J0, 0, 0);
    if (C::NT > 1) {
      a_issue(J0, 1, 1);
    } else {
      const JobInfo J1 = next_job(J0);
      a_issue(J1, 0, 1);
      halo_issue(J1, 1, 0, C::NHQ);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  epi_pre |= dbg;
  int sc = 0;  // global step counter (weight ring position)
  JobInfo J = tile_job(tile0);
  JobInfo J1 = next_job(J);
  JobInfo J2 = C::NT > 1 ? J1 : next_job(J1);
  for (int j = 0;; ++j) {
    if (j > 0) {  // slide the job window
      J = J1;
      if (C::NT > 1) {
        J1 = next_job(J1);
        J2 = J1;
      } else {
        J1 = J2;
        J2 = next_job(J2);
      }
    }
    if (!J.valid) break;
    const int hb = j % C::NH;
    int tuse[TM];  // PH4: taps (bit t = i*2 + j) accumulator block i multiplies
    if constexpr (PH4) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int q = (J.c0 + wc * 32 * TM + 32 * i) / p.phc;
        tuse[i] = 1 | (ph4_b(q) ? 2 : 0) | (ph4_a(q) ? 4 : 0) | (ph4_a(q) && ph4_b(q) ? 8 : 0);
      }
    }
    if (J.k == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][b][e] = 0.f;
    }
    const char* H = Hs + hb * C::HSZ + b_base;
#pragma unroll
    for (int t = 0; t < C::NT; ++t, ++sc) {
      const int ti = t / TW, tj = t % TW;
      const char* A = As + (sc % C::NA) * C::ASZ;
      // loads issued in this step: weights of step sc+2, halo of a later job
      const JobInfo& JA = t + 2 < C::NT ? J : (C::NT > 1 ? J1 : J2);
      const int ta = t + 2 < C::NT ? t + 2 : (C::NT > 1 ? t + 2 - C::NT : 0);
      constexpr bool kNT1 = C::NT == 1;
      const bool do_h = kNT1 || C::q1(t) > C::q0(t);
      const int issued = C::NAQ + (kNT1 ? C::NHQ : C::q1(t) - C::q0(t));

      i32x4 af[2][TM], bfr[2][2];
      auto frag_load = [&](int s, int fb) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[fb][i] = *(const i32x4*)(A + a_off[s] + i * 32 * 128);
#pragma unroll
        for (int b = 0; b < 2; ++b) bfr[fb][b] = *(const i32x4*)(H + (ti * C::HWD + 32 * b + tj) * C::PITCH + s * 32);
      };
      frag_load(0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s < 3) frag_load(s + 1, (s + 1) & 1);
        // DMA issue is spread between the MFMA groups
        if (s == 0) a_issue(JA, ta, (sc + 2) % C::NA);
        if (s == 1 && do_h) {
          if (C::NT > 1)
            halo_issue(J1, (j + 1) % C::NH, C::q0(t), C::q1(t));
          else
            halo_issue(J2, (j + 2) % C::NH, 0, C::NHQ);
        }
        if (PRE && s == 1 && t == PRE_T && J.k + 1 == nchunks) epi_prefetch(J);
        __builtin_amdgcn_sched_barrier(0);
        const int fb = s & 1;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (PH4) {
            if (!((tuse[i] >> t) & 1)) continue;  // (wave-uniform)
          }
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[i][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[fb][i]),
                                                                __builtin_bit_cast(bf16x8, bfr[fb][b]), acc[i][b], 0,
                                                                0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // everything issued before this step has landed (this step's loads may stay in flight;
      // the epilogue prefetch, issued last, too).  Relaxed (epi_pre bit 2, default): the
      // previous step's tail -- its share of the next job's halo and the epilogue prefetch,
      // issued after its weights -- may stay in flight one more step (vmcnt is in order: the
      // older weights of step sc+1 are still waited for), so those HBM/MALL loads get two
      // steps of cover instead of one; at the job's last tap the halo must have landed.
      const bool last = J.k + 1 == nchunks;
      int allow = issued + (PRE && t == PRE_T && last ? npre : 0);
      if (!kNT1 && (epi_pre & 4) && t > 0) {
        const int pre_prev = PRE && t - 1 == PRE_T && last ? npre : 0;
        allow += pre_prev + (t == C::NT - 1 ? 0 : C::q1(t - 1) - C::q0(t - 1));
      }
      wait_vmcnt(allow);
      // plain s_barrier: __syncthreads() would add a release fence, i.e. vmcnt(0)
      __builtin_amdgcn_s_barrier();
    }
    if (J.k + 1 < nchunks) continue;

    // ---- epilogue straight from the accumulators ----
    // permlane32_swap pairs the half-waves so that each lane owns 8 consecutive channels
    // of one pixel: lane half h ends with channels 16P + 8h .. +7 of pair P.
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float v[2][8];
#pragma unroll
        for (int P = 0; P < 2; ++P)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][b][8 * P + e]),
                                                             __float_as_uint(acc[i][b][8 * P + 4 + e]), false, false);
            v[P][e] = __uint_as_float(sw[0]);
            v[P][4 + e] = __uint_as_float(sw[1]);
          }
        const int oy = J.y0 + wp, ox = J.x0 + 32 * b + r32;
        if (oy >= p.oh || ox >= p.ow) continue;
        // output placement (identity, or a stride phase of the strided data gradient)
        long long pix = ((long long)J.n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
        int cq = 0;  // PH4: first channel of this block's phase
        if constexpr (PH4) {
          const int q = (J.c0 + wc * 32 * TM + 32 * i) / p.phc, a = ph4_a(q), pb = ph4_b(q);
          if (2 * oy + a >= p.yh || 2 * ox + pb >= p.yw) continue;
          pix += (long long)a * p.yw + pb;
          cq = q * p.phc;
        }
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          const int co = J.c0 + wc * 32 * TM + 32 * i + 16 * P + 8 * hh - cq;
          if (co + cq >= p.cout) continue;
          float* w = v[P];
          if (p.bias) {
            const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[e] += b0[e];
              w[4 + e] += b1[e];
            }
          }
          if constexpr (OUTF32) {
            float* dst = (float*)p.y + pix * p.y_ld + co;
            if (p.res) {
              const float* rs = (const float*)p.res + pix * p.res_ld + co;
              const f32x4 r0 = *(const f32x4*)rs, r1 = *(const f32x4*)(rs + 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[e] += r0[e];
                w[4 + e] += r1[e];
              }
            }
            if (p.beta) {
              const f32x4 r0 = *(const f32x4*)dst, r1 = *(const f32x4*)(dst + 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[e] += r0[e];
                w[4 + e] += r1[e];
              }
            }
            act_apply<true>(w, 8, p.act, p.alpha);
            if (p.dact) {
              float z[8];
              const i32x4 tz = *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                z[2 * e] = __uint_as_float(((uint32_t)tz[e]) << 16);
                z[2 * e + 1] = __uint_as_float(((uint32_t)tz[e]) & 0xffff0000u);
              }
              dact_apply(w, z, 8, p.dact, p.alpha);
            }
            *(f32x4*)dst = f32x4{w[0], w[1], w[2], w[3]};
            *(f32x4*)(dst + 4) = f32x4{w[4], w[5], w[6], w[7]};
          } else {
            bf16_t* dst = (bf16_t*)p.y + pix * p.y_ld + co;
            if (p.res) {
              const i32x4 tr = PRE ? pre_r[i][b][P] : *(const i32x4*)((const bf16_t*)p.res + pix * p.res_ld + co);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[2 * e] += __uint_as_float(((uint32_t)tr[e]) << 16);
                w[2 * e + 1] += __uint_as_float(((uint32_t)tr[e]) & 0xffff0000u);
              }
            }
            if (p.beta) {
              const i32x4 tr = PRE ? pre_b[i][b][P] : *(const i32x4*)dst;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[2 * e] += __uint_as_float(((uint32_t)tr[e]) << 16);
                w[2 * e + 1] += __uint_as_float(((uint32_t)tr[e]) & 0xffff0000u);
              }
            }
            act_apply(w, 8, p.act, p.alpha);
            if (p.dact) {
              float z[8];
              const i32x4 tz = PRE ? pre_z[i][b][P] : *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                z[2 * e] = __uint_as_float(((uint32_t)tz[e]) << 16);
                z[2 * e + 1] = __uint_as_float(((uint32_t)tz[e]) & 0xffff0000u);
              }
              dact_apply(w, z, 8, p.dact, p.alpha);
            }
            i32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (int)pack_bf16x2(w[2 * e], w[2 * e + 1]);
            *(i32x4*)dst = o;
          }
        }
      }
  }
}

// DVIE_EPI_PREFETCH=0: epilogue operands loaded in the epilogue (A/B runs)
static const bool epi_prefetch_on = !(getenv("DVIE_EPI_PREFETCH") && *getenv("DVIE_EPI_PREFETCH") == '0');
static const int halo_setprio = getenv("DVIE_SETPRIO") && *getenv("DVIE_SETPRIO") == '1' ? 2 : 0;
// DVIE_HALO_WAIT=0: every step waits for all loads issued before it (A/B runs); read per launch
static int halo_wait_flag() {
  const char* e = getenv("DVIE_HALO_WAIT");
#ifdef DVIE_TIMING_DBG
  const char* d = getenv("DVIE_HALO_DBG");  // timing experiments only: 8 = no weight, 16 = no halo streaming
  return (e && *e == '0' ? 0 : 4) | (d && *d ? (atoi(d) & 24) : 0);
#else
  return e && *e == '0' ? 0 : 4;
#endif
}

template <int TM, int WC, int WP, int TH, int TW, bool PH4 = false>
static bool try_halo(const dvie_conv_desc& p, hipStream_t s) {
  typedef HaloCfg<TM, WC, WP, TH, TW> C;
  if constexpr (C::SMEM > 163840) {
    return false;
  } else {
    const int n_ct = (p.cout + C::BC - 1) / C::BC;
    const int tiles_x = (p.ow + 63) / 64, tiles_y = (p.oh + C::PR - 1) / C::PR;
    const long long nt = (long long)n_ct * tiles_x * tiles_y * p.n;
    if (nt >= (1LL << 30)) return false;
    const int n_tiles = (int)nt;
    const int per_cu = 163840 / C::SMEM;
    const int cap = 256 * (per_cu > 2 ? 2 : per_cu);
    const int persistent = n_tiles > cap ? 1 : 0;
    const int grid = persistent ? cap : n_tiles;
    if constexpr (PH4)
      DVIE_LAUNCH((conv_halo_kernel<TM, WC, WP, TH, TW, false, true>), dim3(grid), dim3(C::NTH), 0, s, p, n_ct,
                  n_tiles, tiles_x, tiles_y, persistent, (epi_prefetch_on ? 1 : 0) | halo_setprio | halo_wait_flag());
    else if (p.out_f32)
      DVIE_LAUNCH((conv_halo_kernel<TM, WC, WP, TH, TW, true>), dim3(grid), dim3(C::NTH), 0, s, p, n_ct,
                         n_tiles, tiles_x, tiles_y, persistent, halo_setprio | halo_wait_flag());
    else
      DVIE_LAUNCH((conv_halo_kernel<TM, WC, WP, TH, TW, false>), dim3(grid), dim3(C::NTH), 0, s, p, n_ct,
                         n_tiles, tiles_x, tiles_y, persistent, (epi_prefetch_on ? 1 : 0) | halo_setprio | halo_wait_flag());
    return true;
  }
}

// tile configurations: id -> (TM, WC, WP): BC = 32*TM*WC output channels x WP rows x 64 pixels,
// WC*WP waves
template <int TH, int TW>
static bool launch_cfg(int cfg, const dvie_conv_desc& p, hipStream_t s) {
  switch (cfg) {
    case 0: return try_halo<2, 1, 4, TH, TW>(p, s);  // 64 co x 4 rows, 4 waves
    case 1: return try_halo<2, 2, 2, TH, TW>(p, s);  // 128 co x 2 rows, 4 waves
    case 2: return try_halo<1, 1, 4, TH, TW>(p, s);  // 32 co x 4 rows, 4 waves
    case 3: return try_halo<1, 2, 4, TH, TW>(p, s);  // 64 co x 4 rows, 8 waves
    case 4: return try_halo<2, 2, 4, TH, TW>(p, s);  // 128 co x 4 rows, 8 waves
    case 5: return try_halo<1, 4, 2, TH, TW>(p, s);  // 128 co x 2 rows, 8 waves
    case 6: return try_halo<1, 1, 8, TH, TW>(p, s);  // 32 co x 8 rows, 8 waves
    case 7: return try_halo<2, 1, 8, TH, TW>(p, s);  // 64 co x 8 rows, 8 waves
  }
  return false;
}

template <int TH, int TW>
static bool launch_cfg2(int cfg, const dvie_conv_desc& p, hipStream_t s) {
  return cfg == 3 ? try_halo<1, 2, 4, TH, TW>(p, s) : try_halo<2, 2, 4, TH, TW>(p, s);
}

static int env_cfg() {
  // tuning override (read per launch so a tuner can sweep it in one process):
  // -1 = per-tap kernel (conv_fwd.hip), 0..4 = halo configuration, unset = automatic
  const char* e = getenv("DVIE_CONV_CFG");
  return e && *e ? atoi(e) : -3;
}

// Epilogue of one 32-channel x 32-pixel accumulator block (v_mfma_f32_32x32x16 layout):
// permlane32_swap pairs the half-waves so that each lane owns 8 consecutive channels of one
// pixel, then bias / residual / accumulate / activation / activation-derivative and one
// 16-byte (bf16) or 2x16-byte (fp32) store per lane.  co8 = the lane's first channel of
// pair 0 (32-block base + 8 * half); pair P adds 16.
template <bool OUTF32>
__device__ __forceinline__ void ws_epilogue(const dvie_conv_desc& p, const f32x16& acc, int n, int oy, int ox, int co8) {
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
  if (oy >= p.oh || ox >= p.ow) return;
  const long long pix = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
#pragma unroll
  for (int P = 0; P < 2; ++P) {
    const int co = co8 + 16 * P;
    if (co >= p.cout) continue;
    float* w = v[P];
    if (p.bias) {
      const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w[e] += b0[e];
        w[4 + e] += b1[e];
      }
    }
    float t8[8];
    if constexpr (OUTF32) {
      float* dst = (float*)p.y + pix * p.y_ld + co;
      if (p.res) {
        const float* rs = (const float*)p.res + pix * p.res_ld + co;
        const f32x4 r0 = *(const f32x4*)rs, r1 = *(const f32x4*)(rs + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[e] += r0[e];
          w[4 + e] += r1[e];
        }
      }
      if (p.beta) {
        const f32x4 r0 = *(const f32x4*)dst, r1 = *(const f32x4*)(dst + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[e] += r0[e];
          w[4 + e] += r1[e];
        }
      }
      act_apply<true>(w, 8, p.act, p.alpha);
      if (p.dact) {
        const i32x4 tz = *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t8[2 * e] = __uint_as_float(((uint32_t)tz[e]) << 16);
          t8[2 * e + 1] = __uint_as_float(((uint32_t)tz[e]) & 0xffff0000u);
        }
        dact_apply(w, t8, 8, p.dact, p.alpha);
      }
      *(f32x4*)dst = f32x4{w[0], w[1], w[2], w[3]};
      *(f32x4*)(dst + 4) = f32x4{w[4], w[5], w[6], w[7]};
    } else {
      bf16_t* dst = (bf16_t*)p.y + pix * p.y_ld + co;
      if (p.res) {
        const i32x4 tr = *(const i32x4*)((const bf16_t*)p.res + pix * p.res_ld + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[2 * e] += __uint_as_float(((uint32_t)tr[e]) << 16);
          w[2 * e + 1] += __uint_as_float(((uint32_t)tr[e]) & 0xffff0000u);
        }
      }
      if (p.beta) {
        const i32x4 tr = *(const i32x4*)dst;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[2 * e] += __uint_as_float(((uint32_t)tr[e]) << 16);
          w[2 * e + 1] += __uint_as_float(((uint32_t)tr[e]) & 0xffff0000u);
        }
      }
      act_apply(w, 8, p.act, p.alpha);
      if (p.dact) {
        const i32x4 tz = *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t8[2 * e] = __uint_as_float(((uint32_t)tz[e]) << 16);
          t8[2 * e + 1] = __uint_as_float(((uint32_t)tz[e]) & 0xffff0000u);
        }
        dact_apply(w, t8, 8, p.dact, p.alpha);
      }
      i32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (int)pack_bf16x2(w[2 * e], w[2 * e + 1]);
      *(i32x4*)dst = o;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Weight-stationary variant for single-chunk 3x3 convs (c <= 64, cout <= 64: the 64-channel
// full-resolution HRNet branch, its data gradient, VGG conv1_2): every wave keeps the
// weights of its 32 output channels for all 9 taps in VGPRs (loaded once per workgroup), so
// the tap loop reads only input-halo fragments from LDS and needs no barrier; one barrier
// per output tile (halo double buffer).  8 waves = 2 channel halves x 4 output rows.
// WP = output rows per tile: 4 (8 waves, one workgroup per CU) or 2 (4 waves, two
// workgroups per CU: twice the independent halo streams in flight per CU).
template <int KS, bool OUTF32, int WP>
__global__ __launch_bounds__(2 * WP * 64, 4 / WP) void conv_ws_kernel(const dvie_conv_desc p, int n_tiles,
                                                                       int tiles_x, int tiles_y, int persistent) {
  typedef HaloCfg<1, 2, WP, 3, 3> C;  // halo geometry of a WP-row x 64-pixel tile, 2*WP waves
  constexpr int NW = 2 * WP;
  __shared__ __attribute__((aligned(1024))) char smem[2 * C::HSZ];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / WP, wp = wave % WP;
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  int tile0, tile_end, tile_step;
  if (!persistent) {
    tile0 = xcd_remap3(blockIdx.x, n_tiles);
    tile_end = tile0 + 1;
    tile_step = 1;
  } else {
    const int G = gridDim.x, g = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int nbg = G / 8 + (g < G % 8 ? 1 : 0);
    const int q = n_tiles / 8, r = n_tiles % 8;
    const int ts = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
    tile0 = ts + j;
    tile_end = ts + q + (g < r ? 1 : 0);
    tile_step = nbg;
  }
  if (tile0 >= tile_end) return;

  // ---- weights -> VGPRs: lane (r32, h) holds w[co][t*c + 16s + 8h .. +7], co = 32*wc + r32
  i32x4 wa[9][KS];
  {
    const int co = 32 * wc + r32;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int sl = 0; sl < KS; ++sl) {
        const int k = 16 * sl + 8 * hh;
        i32x4 v = {0, 0, 0, 0};
        if (co < p.cout && k < p.c) v = *(const i32x4*)((const bf16_t*)p.w + (long long)co * p.kpad + t * p.c + k);
        wa[t][sl] = v;
      }
  }

  int hgeo[C::NHQ];
#pragma unroll
  for (int q = 0; q < C::NHQ; ++q) {
    const int slot = (wave + NW * q) * 64 + lane;
    const int hr = slot / 9, cs = slot - 9 * (slot / 9);
    const int hy = hr / C::HWD, hx = hr - (hr / C::HWD) * C::HWD;
    hgeo[q] = (cs < 8 && cs * 8 < p.c && hr < C::HR * C::HWD) ? (hy << 16) | (hx << 4) | cs : -1;
  }
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)xbytes, 0x00020000);

  struct TP {
    int n, y0, x0;
  };
  auto decode = [&](int t) {
    TP q;
    q.x0 = (t % tiles_x) * 64;
    const int r = t / tiles_x;
    q.y0 = (r % tiles_y) * C::PR;
    q.n = r / tiles_y;
    return q;
  };
  auto halo_issue = [&](const TP& T, int hb) {
    char* dst = smem + hb * C::HSZ + wave * 1024;
    const int ybase = T.y0 + p.dy0, xbase = T.x0 + p.dx0;
#pragma unroll
    for (int q = 0; q < C::NHQ; ++q) {
      const int gq = hgeo[q];
      const int iy = ybase + (gq >> 16), ix = xbase + ((gq >> 4) & 0xFFF);
      const bool ok = gq >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
      const unsigned o = ok ? (unsigned)((T.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(gq & 15) * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(dst + q * NW * 1024), 16, o, 0, 0, 0);
    }
  };

  const int b_base = (wp * C::HWD + r32) * C::PITCH + hh * 16;
  TP cur = decode(tile0);
  halo_issue(cur, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  int hb = 0;
  for (int tile = tile0; tile < tile_end; tile += tile_step, hb ^= 1) {
    const bool has_next = tile + tile_step < tile_end;
    const TP nxt = decode(has_next ? tile + tile_step : tile);
    if (has_next) halo_issue(nxt, hb ^ 1);

    f32x16 acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    const char* H = smem + hb * C::HSZ + b_base;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ti = t / 3, tj = t % 3;
#pragma unroll
      for (int sl = 0; sl < KS; ++sl) {
        i32x4 bf[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[b] = *(const i32x4*)(H + (ti * C::HWD + 32 * b + tj) * C::PITCH + sl * 32);
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa[t][sl]),
                                                           __builtin_bit_cast(bf16x8, bf[b]), acc[b], 0, 0, 0);
      }
    }
    // the next tile's halo has landed and every wave is done with this one
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();

    // ---- epilogue straight from the accumulators (as conv_halo_kernel) ----
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int oy = cur.y0 + wp, ox = cur.x0 + 32 * b + r32;
      ws_epilogue<OUTF32>(p, acc[b], cur.n, oy, ox, 32 * wc + 8 * hh);
    }
    cur = nxt;
  }
}

template <int KS, int WP>
static void launch_ws_rows(const dvie_conv_desc& p, hipStream_t s) {
  const int tiles_x = (p.ow + 63) / 64, tiles_y = (p.oh + WP - 1) / WP;
  const int n_tiles = tiles_x * tiles_y * p.n;
  const int cap = 256 * (4 / WP);  // resident workgroups: one (WP 4) or two (WP 2) per CU
  const int persistent = n_tiles > cap ? 1 : 0;
  const int grid = persistent ? cap : n_tiles;
  if (p.out_f32)
    DVIE_LAUNCH((conv_ws_kernel<KS, true, WP>), dim3(grid), dim3(2 * WP * 64), 0, s, p, n_tiles, tiles_x,
                       tiles_y, persistent);
  else
    DVIE_LAUNCH((conv_ws_kernel<KS, false, WP>), dim3(grid), dim3(2 * WP * 64), 0, s, p, n_tiles, tiles_x,
                       tiles_y, persistent);
}

// tuning knob (read once): DVIE_WS_ROWS = 2 (default: two workgroups per CU, +1.3% step
// same-box A/B 192.8-193.1 vs 190.5 frames/s, profiles/r02_ab/ab_wsrows.txt) or 4
static const int ws_rows = getenv("DVIE_WS_ROWS") && atoi(getenv("DVIE_WS_ROWS")) == 4 ? 4 : 2;

template <int KS>
static void launch_ws(const dvie_conv_desc& p, hipStream_t s) {
  if (ws_rows == 2)
    launch_ws_rows<KS, 2>(p, s);
  else
    launch_ws_rows<KS, 4>(p, s);
}

// ---------------------------------------------------------------------------------------
// Strip variant of the weight-stationary 3x3 conv (c <= 64, cout <= 64).  conv_ws_kernel
// stages a (WP+2)-row halo per WP output rows, so every input row is fetched 1.5-2x, and it
// prefetches one tile ahead, which does not cover HBM latency at two waves per SIMD.  Here a
// workgroup owns a 64-pixel column strip of a segment of SEG output rows and walks down it:
// the input rows live in an LDS ring, each row is fetched ONCE per segment (row overhead
// (SEG+2)/SEG, column overhead 66/64), and the rows of iteration i+D are issued at the start
// of iteration i, D iterations of MFMA work ahead of their use.
// * Ring row: 66 pixels x 144 B (8 data slots + 1 pad slot, conflict-free tap-shifted
//   ds_read_b128 as in the halo kernels), filled by 10 LDS-DMA pieces of 1 KiB.
// * Iteration i computes output rows i*WR .. i*WR+WR-1 of the segment (one per row-wave,
//   two channel halves of 32), from ring rows i*WR .. i*WR+WR+1.  Group i loads rows
//   i*WR+2 .. i*WR+WR+1 (the two leading rows are a prologue group), so with
//   RR = WR+2+D*WR ring rows, group i+D overwrites only rows of iterations < i.
// * One barrier per iteration: after it, every wave's DMA of group i has landed and every
//   wave is done with iteration i-1.  Groups past the segment end are issued against an
//   empty buffer range (no traffic), so every wave's vmcnt bookkeeping is compile-time.
template <int WR, int D>
struct StripCfg {
  static constexpr int NW = 2 * WR;
  static constexpr int HWD = 66, PITCH = 144;
  static constexpr int RP = (HWD * 9 + 63) / 64;        // DMA pieces per ring row (10)
  static constexpr int RB = RP * 1024;                   // bytes per ring row
  static constexpr int RR = WR + 2 + D * WR;             // ring rows
  static constexpr int NPL = RP * WR / NW;               // pieces per wave per group (5)
  static constexpr int NP0 = (2 * RP + NW - 1) / NW;     // pieces per wave, prologue rows
  static constexpr int JUNK = NP0 * NW - 2 * RP;         // prologue pieces with no row
  static constexpr int SMEM = RR * RB + JUNK * 1024;
  static_assert(RP * WR % NW == 0, "uniform pieces per wave");
};

// bf16 epilogue of one 32x32 accumulator block from operands prefetched into registers
// (EPI: 1 residual, 2 accumulate target, 4 activation input; i32x4 [pair P] each)
template <int EPI>
__device__ __forceinline__ void strip_epilogue(const dvie_conv_desc& p, const f32x16& acc, int n, int oy, int ox, int co8,
                                               const i32x4* er, const i32x4* eb, const i32x4* ez) {
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
  if (oy >= p.oh || ox >= p.ow) return;
  const long long pix = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
#pragma unroll
  for (int P = 0; P < 2; ++P) {
    const int co = co8 + 16 * P;
    if (co >= p.cout) continue;
    float* w = v[P];
    if (p.bias) {
      const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w[e] += b0[e];
        w[4 + e] += b1[e];
      }
    }
    auto add_bf = [&](const i32x4 t) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w[2 * e] += __uint_as_float(((uint32_t)t[e]) << 16);
        w[2 * e + 1] += __uint_as_float(((uint32_t)t[e]) & 0xffff0000u);
      }
    };
    if constexpr ((EPI & 1) != 0) add_bf(er[P]);
    if constexpr ((EPI & 2) != 0) add_bf(eb[P]);
    act_apply(w, 8, p.act, p.alpha);
    if constexpr ((EPI & 4) != 0) {
      float z[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        z[2 * e] = __uint_as_float(((uint32_t)ez[P][e]) << 16);
        z[2 * e + 1] = __uint_as_float(((uint32_t)ez[P][e]) & 0xffff0000u);
      }
      dact_apply(w, z, 8, p.dact, p.alpha);
    }
    i32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (int)pack_bf16x2(w[2 * e], w[2 * e + 1]);
    *(i32x4*)((bf16_t*)p.y + pix * p.y_ld + co) = o;
  }
}

// EPI < 0: fp32 output, operands read in the epilogue (parity mode, not tuned)
template <int KS, int EPI, int WR, int D>
__global__ __launch_bounds__(2 * WR * 64, 4 / WR) void conv_strip_kernel(const dvie_conv_desc p, int tiles_x, int nseg,
                                                                          int seg, int n_wg) {
  typedef StripCfg<WR, D> C;
  constexpr int NW = C::NW;
  constexpr bool OUTF32 = EPI < 0;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / WR, wr = wave % WR;
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // logical id: segments of one strip consecutive (they share boundary rows in L2)
  const int lid = xcd_remap3(blockIdx.x, n_wg);
  const int sg = lid % nseg;
  const int strip = (lid / nseg) % tiles_x;
  const int n = lid / nseg / tiles_x;
  const int ys = sg * seg, x0 = strip * 64;
  if (ys >= p.oh) return;
  const int niter = (min(seg, p.oh - ys) + WR - 1) / WR;

  // ---- weights -> VGPRs (as conv_ws_kernel)
  i32x4 wa[9][KS];
  {
    const int co = 32 * wc + r32;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int sl = 0; sl < KS; ++sl) {
        const int k = 16 * sl + 8 * hh;
        i32x4 v = {0, 0, 0, 0};
        if (co < p.cout && k < p.c) v = *(const i32x4*)((const bf16_t*)p.w + (long long)co * p.kpad + t * p.c + k);
        wa[t][sl] = v;
      }
  }

  // ---- DMA: piece pc of a group -> (row j in the group, 1-KiB piece pr of the ring row)
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const int xb = x0 + p.dx0, yb = ys + p.dy0;  // input column of ring pixel 0, input row of ring row 0
  auto lane_off = [&](int pr, int iy) -> unsigned {
    const int slot = pr * 64 + lane;
    const int px = slot / 9, cs = slot - 9 * (slot / 9);
    const int ix = xb + px;
    const bool ok = px < C::HWD && cs < 8 && cs * 8 < p.c && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
    return ok ? (unsigned)((n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)cs * 16u : OOB;
  };
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rnone = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, 0, 0x00020000);
  // group g: ring rows R = g*WR+2+j, j < WR (rows past the segment: empty range, no traffic)
  auto group_issue = [&](int g) {
    const __amdgpu_buffer_rsrc_t r = g < niter ? rx : rnone;
#pragma unroll
    for (int q = 0; q < C::NPL; ++q) {
      const int pc = wave + NW * q;
      const int j = pc / C::RP, pr = pc - C::RP * (pc / C::RP);
      const int R = g * WR + 2 + j;
      char* dst = smem + (R % C::RR) * C::RB + pr * 1024;
      // (offset as a separate statement: see halo_issue)
      const unsigned o = lane_off(pr, yb + R);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, o, 0, 0, 0);
    }
  };
  {  // prologue: ring rows 0 and 1 (pieces without a row land in the junk area), groups 0..D-1
#pragma unroll
    for (int q = 0; q < C::NP0; ++q) {
      const int pc = wave + NW * q;
      const int j = pc / C::RP, pr = pc - C::RP * (pc / C::RP);
      char* dst = pc < 2 * C::RP ? smem + j * C::RB + pr * 1024 : smem + C::RR * C::RB + (pc - 2 * C::RP) * 1024;
      const unsigned o = pc < 2 * C::RP ? lane_off(pr, yb + j) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)dst, 16, o, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < D; ++g) group_issue(g);
  }

  // epilogue operands of iteration i, issued before group i+D so that waiting for them never
  // waits for the look-ahead rows
  constexpr int NE = OUTF32 ? 0 : 4 * (((EPI & 1) ? 1 : 0) + ((EPI & 2) ? 1 : 0) + ((EPI & 4) ? 1 : 0));
  i32x4 er[2][2], eb[2][2], ez[2][2];
  auto epi_issue = [&](int i) {
    const int oy = ys + i * WR + wr;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const int ox = x0 + 32 * b + r32, co = 32 * wc + 8 * hh + 16 * P;
        const bool ok = oy < p.oh && ox < p.ow && co < p.cout;
        const long long pix = ((long long)n * p.yh + (long long)oy * p.osy + p.ory) * p.yw + (long long)ox * p.osx + p.orx;
        if constexpr ((EPI & 1) != 0) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p.res, 0, 0x7FFFFFF0, 0x00020000);
          er[b][P] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (unsigned)((pix * p.res_ld + co) * 2) : OOB, 0, 0);
        }
        if constexpr ((EPI & 2) != 0) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p.y, 0, 0x7FFFFFF0, 0x00020000);
          eb[b][P] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (unsigned)((pix * p.y_ld + co) * 2) : OOB, 0, 0);
        }
        if constexpr ((EPI & 4) != 0) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, 0, 0x7FFFFFF0, 0x00020000);
          ez[b][P] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (unsigned)((pix * p.z_ld + co) * 2) : OOB, 0, 0);
        }
      }
  };

  constexpr int NST = OUTF32 ? 8 : 4;  // epilogue stores per wave per iteration (at most)
  const int b_lane = r32 * C::PITCH + hh * 16;
  for (int i = 0; i < niter; ++i) {
    // groups <= i landed; in flight may stay: groups i+1 .. i+D-1, the stores of the last
    // min(i, D) iterations, the epilogue operands of the last min(i, D-1) iterations
    wait_vmcnt((D - 1) * C::NPL + min(i, D) * NST + min(i, D - 1) * NE);
    __builtin_amdgcn_s_barrier();
    if constexpr (NE > 0) epi_issue(i);
    group_issue(i + D);

    f32x16 acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
#pragma unroll
    for (int ti = 0; ti < 3; ++ti) {
      const char* H = smem + ((i * WR + wr + ti) % C::RR) * C::RB + b_lane;
#pragma unroll
      for (int tj = 0; tj < 3; ++tj)
#pragma unroll
        for (int sl = 0; sl < KS; ++sl) {
          i32x4 bf[2];
#pragma unroll
          for (int b = 0; b < 2; ++b) bf[b] = *(const i32x4*)(H + (32 * b + tj) * C::PITCH + sl * 32);
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa[3 * ti + tj][sl]),
                                                             __builtin_bit_cast(bf16x8, bf[b]), acc[b], 0, 0, 0);
        }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if constexpr (OUTF32)
        ws_epilogue<true>(p, acc[b], n, ys + i * WR + wr, x0 + 32 * b + r32, 32 * wc + 8 * hh);
      else
        strip_epilogue<(EPI < 0 ? 0 : EPI)>(p, acc[b], n, ys + i * WR + wr, x0 + 32 * b + r32, 32 * wc + 8 * hh, er[b], eb[b],
                                          ez[b]);
    }
  }
  // drain: no DMA may still target this workgroup's LDS when it exits
  __builtin_amdgcn_s_waitcnt(0);
}

template <int KS, int WR, int D, int EPI>
static void launch_strip_k(const dvie_conv_desc& p, hipStream_t s) {
  const int tiles_x = (p.ow + 63) / 64;
  const int cap = 256 * (4 / WR);  // resident workgroups
  const int cols = p.n * tiles_x;
  int nseg = cap / cols;
  if (nseg < 1) nseg = 1;
  if (nseg > (p.oh + WR - 1) / WR) nseg = (p.oh + WR - 1) / WR;
  int seg = (p.oh + nseg - 1) / nseg;
  seg = (seg + WR - 1) / WR * WR;
  nseg = (p.oh + seg - 1) / seg;
  const int n_wg = cols * nseg;
  DVIE_LAUNCH((conv_strip_kernel<KS, EPI, WR, D>), dim3(n_wg), dim3(2 * WR * 64), 0, s, p, tiles_x, nseg, seg,
                     n_wg);
}

// epilogue-operand set of a launch -> kernel instance (fp32 output: EPI -1)
// (all three operands: not taken -- their registers do not fit next to the weights)
template <int KS, int WR, int D>
static bool launch_strip_cfg(const dvie_conv_desc& p, hipStream_t s) {
  if (p.out_f32) {
    launch_strip_k<KS, WR, D, -1>(p, s);
    return true;
  }
  switch ((p.res ? 1 : 0) | (p.beta ? 2 : 0) | (p.dact ? 4 : 0)) {
    case 0: launch_strip_k<KS, WR, D, 0>(p, s); return true;
    case 1: launch_strip_k<KS, WR, D, 1>(p, s); return true;
    case 2: launch_strip_k<KS, WR, D, 2>(p, s); return true;
    case 3: launch_strip_k<KS, WR, D, 3>(p, s); return true;
    case 4: launch_strip_k<KS, WR, D, 4>(p, s); return true;
    case 5: launch_strip_k<KS, WR, D, 5>(p, s); return true;
    case 6: launch_strip_k<KS, WR, D, 6>(p, s); return true;
  }
  return false;
}

// DVIE_CONV_STRIP: 0 = conv_ws_kernel (A/B runs); 1 = strip, 4 rows per iteration, 2
// iterations ahead (one 8-wave workgroup per CU); 2 (default) = strip, 2 rows, 2 ahead (two
// 4-wave workgroups per CU); 3 = strip, 2 rows, 1 ahead.  Read per launch (tuning sweeps).
// Measured (tools/conv_strip_micro.py, profiles/r02_ab/conv_strip_micro.txt), 8x256x512
// 64->64: tile kernel / mode 2 = 96 / 96 us plain, 138 / 108 residual, 130 / 111 activation
// input, 159 / 130 accumulate + activation input.
static int strip_mode() {
  const char* e = getenv("DVIE_CONV_STRIP");
  return e && *e ? atoi(e) : 2;
}

template <int KS>
static bool launch_strip(const dvie_conv_desc& p, hipStream_t s) {
  switch (strip_mode()) {
    case 1: return launch_strip_cfg<KS, 4, 2>(p, s);
    case 2: return launch_strip_cfg<KS, 2, 2>(p, s);
    case 3: return launch_strip_cfg<KS, 2, 1>(p, s);
  }
  return false;
}

// ---------------------------------------------------------------------------------------
// Dense-K variant for 3x3 stride-1 convs with few input channels (c = 8, 16 or 24: the data
// gradients of the 3- / 20-channel output heads into their 448-channel hidden layers, the
// 20-channel seg encoder, the image stems).  The chunked kernels give every tap a 64-channel
// K slice, so c = 8 spends 7/8 of its MFMAs on zeros.  Here K is the flattened (tap,
// channel) axis of the packed weights, 9c long: a 16-deep MFMA slice covers two 8-channel
// groups -- lane half h takes group 2s + h, i.e. its own tap -- so c = 8 needs 5 slices per
// output block instead of 36 (c = 24: 14 instead of 36).
// * Halo image: CP8 = c/8 slots of 16 B per pixel (pitch 16 B for c = 8, 48 B otherwise: a
//   16-lane ds_read_b128 group then touches 16 distinct bank quads), LDS-DMA filled,
//   double-buffered; ~6-19 KB per tile, so several workgroups share a CU.
// * A workgroup owns one 64-channel output block (weights in VGPRs for all slices, loaded
//   once) and walks output tiles of 4 rows x 64 pixels; 8 waves = 2 channel halves x 4 rows.
//   Workgroups of one tile (one per output block) are consecutive logical ids on one XCD,
//   so the halo is read from HBM once and from L2 by the others.
template <int CP8>
struct NkCfg {
  static constexpr int WP = 4, NW = 8;
  static constexpr int HR = WP + 2, HWD = 66;
  static constexpr int PS = CP8 == 1 ? 1 : 3;  // 16-B slots per pixel (pitch)
  static constexpr int SLOTS = HR * HWD * PS;
  static constexpr int NPC = ((SLOTS + 63) / 64 + NW - 1) / NW;  // DMA pieces per wave
  static constexpr int HSZ = NPC * NW * 1024;
  static constexpr int NG = 9 * CP8;         // 8-channel groups along K
  static constexpr int NS = (NG + 1) / 2;    // 16-deep MFMA slices
};

template <int CP8, bool OUTF32, bool PRE = false>
__global__ __launch_bounds__(512, 2) void conv_nk_kernel(const dvie_conv_desc p, int n_cb, int n_tiles, int tiles_x,
                                                        int tiles_y) {
  typedef NkCfg<CP8> C;
  __shared__ __attribute__((aligned(1024))) char smem[2 * C::HSZ];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / C::WP, wp = wave % C::WP;
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // logical id: (tile-major, output block fastest), XCD-contiguous ranges
  const int lid = xcd_remap3(blockIdx.x, gridDim.x);
  const int cb = lid % n_cb;
  const int per_cb = gridDim.x / n_cb;  // workgroups per output block (grid = n_cb * per_cb)
  const int tile0 = lid / n_cb;
  if (tile0 >= n_tiles) return;

  // weights -> VGPRs: lane (r32, h) holds w[co][16 s + 8 h .. +7] of the flattened K = 9c
  i32x4 wa[C::NS];
  {
    const int co = cb * 64 + 32 * wc + r32;
#pragma unroll
    for (int sl = 0; sl < C::NS; ++sl) {
      const int k = 16 * sl + 8 * hh;
      i32x4 v = {0, 0, 0, 0};
      if (co < p.cout && k < 9 * p.c) v = *(const i32x4*)((const bf16_t*)p.w + (long long)co * p.kpad + k);
      wa[sl] = v;
    }
  }
  // B fragment offsets: group g = 2 s + h -> tap t = g / CP8 (row t/3, column t%3), 16-B
  // slot g % CP8 of the shifted pixel
  int boff[C::NS];
#pragma unroll
  for (int sl = 0; sl < C::NS; ++sl) {
    const int g = 2 * sl + hh;
    const int t = g < C::NG ? g / CP8 : 0, j = g < C::NG ? g % CP8 : 0;
    boff[sl] = (((t / 3) * C::HWD + (t % 3)) * C::PS + j) * 16;
  }
  // DMA geometry: slot -> (halo row, halo column, 16-B channel group)
  int hgeo[C::NPC];
#pragma unroll
  for (int q = 0; q < C::NPC; ++q) {
    const int slot = (wave + C::NW * q) * 64 + lane;
    const int px = slot / C::PS, cs = slot - C::PS * (slot / C::PS);
    const int hy = px / C::HWD, hx = px - (px / C::HWD) * C::HWD;
    hgeo[q] = (cs < CP8 && cs * 8 < p.c && px < C::HR * C::HWD) ? (hy << 16) | (hx << 4) | cs : -1;
  }
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)xbytes, 0x00020000);
  struct TP {
    int n, y0, x0;
  };
  auto decode = [&](int t) {
    TP q;
    q.x0 = (t % tiles_x) * 64;
    const int r = t / tiles_x;
    q.y0 = (r % tiles_y) * C::WP;
    q.n = r / tiles_y;
    return q;
  };
  auto halo_issue = [&](const TP& T, int hb) {
    char* dst = smem + hb * C::HSZ + wave * 1024;
    const int ybase = T.y0 + p.dy0, xbase = T.x0 + p.dx0;
#pragma unroll
    for (int q = 0; q < C::NPC; ++q) {
      const int gq = hgeo[q];
      const int iy = ybase + (gq >> 16), ix = xbase + ((gq >> 4) & 0xFFF);
      const bool ok = gq >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
      const unsigned o = ok ? (unsigned)((T.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(gq & 15) * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(dst + q * C::NW * 1024), 16, o, 0, 0, 0);
    }
  };

  const int b_base = ((wp * C::HWD + r32) * C::PS) * 16;
  TP cur = decode(tile0);
  halo_issue(cur, 0);
  if constexpr (PRE) {
    // Epilogue operands (residual / accumulate / activation input) of the NEXT tile are loaded
    // into registers right after this tile's stores, and every store and operand load is a
    // buffer instruction that every wave issues (out-of-range lanes aimed past the buffer), so
    // per tile a wave issues exactly [next halo: NPC][stores: 4][operand loads: 4 nops] and the
    // wait before the barrier, vmcnt(4 + 4 nops), covers the halo only: the stores drain and
    // the operands land under the next tile's MFMAs (before: the operands were loaded inside
    // the epilogue and one vmcnt(0) per tile waited for the halo and the stores together).
    const int co0 = cb * 64 + 32 * wc + 8 * hh;
    const unsigned long long yspan =
        ((unsigned long long)p.n * p.yh * p.yw - 1) * (unsigned long long)p.y_ld * 2ull + (unsigned long long)p.cout * 2ull;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.y, 0, (int)yspan, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.res, 0,
        p.res ? (int)(((unsigned long long)p.n * p.yh * p.yw - 1) * (unsigned long long)p.res_ld * 2ull + p.cout * 2ull) : 0,
        0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.z, 0,
        p.dact ? (int)(((unsigned long long)p.n * p.yh * p.yw - 1) * (unsigned long long)p.z_ld * 2ull + p.cout * 2ull) : 0,
        0x00020000);
    const int nops = (p.res ? 1 : 0) + (p.beta ? 1 : 0) + (p.dact ? 1 : 0);
    // the lane's element offsets of accumulator b, pair P in the three operand images (or OOB)
    auto offs = [&](const TP& T, int b, int P, unsigned& oy_, unsigned& or_, unsigned& oz_) {
      const int oy = T.y0 + wp, ox = T.x0 + 32 * b + r32, co = co0 + 16 * P;
      const bool ok = oy < p.oh && ox < p.ow && co < p.cout;
      const long long pix = ((long long)T.n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
      oy_ = ok ? (unsigned)((pix * p.y_ld + co) * 2) : OOB;
      or_ = ok ? (unsigned)((pix * p.res_ld + co) * 2) : OOB;
      oz_ = ok ? (unsigned)((pix * p.z_ld + co) * 2) : OOB;
    };
    // one i32x4 per (operand, b, P); a flag-off operand is never read (its loads are not issued)
    i32x4 er[2][2], eb[2][2], ez[2][2];
    auto prefetch = [&](const TP& T) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          unsigned o_y, o_r, o_z;
          offs(T, b, P, o_y, o_r, o_z);
          if (p.res) er[b][P] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, o_r, 0, 0));
          if (p.beta) eb[b][P] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, o_y, 0, 0));
          if (p.dact) ez[b][P] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rz, o_z, 0, 0));
        }
    };
    f32x4 bia[2][2];
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      const int co = co0 + 16 * P;
      bia[P][0] = p.bias && co < p.cout ? *(const f32x4*)(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      bia[P][1] = p.bias && co < p.cout ? *(const f32x4*)(p.bias + co + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    prefetch(cur);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    int hb = 0;
    for (int tile = tile0; tile < n_tiles; tile += per_cb, hb ^= 1) {
      const bool has_next = tile + per_cb < n_tiles;
      const TP nxt = decode(has_next ? tile + per_cb : tile);
      halo_issue(nxt, hb ^ 1);  // (a repeat of the current tile at the end: uniform counts)
      f32x16 acc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
      const char* H = smem + hb * C::HSZ + b_base;
#pragma unroll
      for (int sl = 0; sl < C::NS; ++sl) {
        i32x4 bf[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[b] = *(const i32x4*)(H + boff[sl] + 32 * b * C::PS * 16);
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa[sl]), __builtin_bit_cast(bf16x8, bf[b]),
                                                           acc[b], 0, 0, 0);
      }
      // epilogue of the current tile from the prefetched operands: 4 buffer stores per wave
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float v[2][8];
#pragma unroll
        for (int P = 0; P < 2; ++P)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[b][8 * P + e]),
                                                             __float_as_uint(acc[b][8 * P + 4 + e]), false, false);
            v[P][e] = __uint_as_float(sw[0]) + bia[P][0][e];
            v[P][4 + e] = __uint_as_float(sw[1]) + bia[P][1][e];
          }
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          float* w = v[P];
          if (p.res) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[2 * e] += __uint_as_float(((uint32_t)er[b][P][e]) << 16);
              w[2 * e + 1] += __uint_as_float(((uint32_t)er[b][P][e]) & 0xffff0000u);
            }
          }
          if (p.beta) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[2 * e] += __uint_as_float(((uint32_t)eb[b][P][e]) << 16);
              w[2 * e + 1] += __uint_as_float(((uint32_t)eb[b][P][e]) & 0xffff0000u);
            }
          }
          act_apply(w, 8, p.act, p.alpha);
          if (p.dact) {
            float t8[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              t8[2 * e] = __uint_as_float(((uint32_t)ez[b][P][e]) << 16);
              t8[2 * e + 1] = __uint_as_float(((uint32_t)ez[b][P][e]) & 0xffff0000u);
            }
            dact_apply(w, t8, 8, p.dact, p.alpha);
          }
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (int)pack_bf16x2(w[2 * e], w[2 * e + 1]);
          unsigned o_y, o_r, o_z;
          offs(cur, b, P, o_y, o_r, o_z);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), ry, o_y, 0, 0);
        }
      }
      prefetch(nxt);
      // outstanding, oldest first: [next halo][4 stores][4 nops operand loads]
      wait_vmcnt(4 + 4 * nops);
      __builtin_amdgcn_s_barrier();
      cur = nxt;
    }
    __builtin_amdgcn_s_waitcnt(0);
    return;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int hb = 0;
  for (int tile = tile0; tile < n_tiles; tile += per_cb, hb ^= 1) {
    const bool has_next = tile + per_cb < n_tiles;
    const TP nxt = decode(has_next ? tile + per_cb : tile);
    if (has_next) halo_issue(nxt, hb ^ 1);
    f32x16 acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    const char* H = smem + hb * C::HSZ + b_base;
#pragma unroll
    for (int sl = 0; sl < C::NS; ++sl) {
      i32x4 bf[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) bf[b] = *(const i32x4*)(H + boff[sl] + 32 * b * C::PS * 16);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa[sl]), __builtin_bit_cast(bf16x8, bf[b]),
                                                         acc[b], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int b = 0; b < 2; ++b)
      ws_epilogue<OUTF32>(p, acc[b], cur.n, cur.y0 + wp, cur.x0 + 32 * b + r32, cb * 64 + 32 * wc + 8 * hh);
    cur = nxt;
  }
}

// DVIE_NK_PRE=0: the narrow-input kernel loads its epilogue operands inside the epilogue
// (A/B runs); read per launch
static bool nk_pre_on() {
  const char* e = getenv("DVIE_NK_PRE");
  return !(e && *e == '0');
}

template <int CP8>
static void launch_nk(const dvie_conv_desc& p, hipStream_t s) {
  typedef NkCfg<CP8> C;
  const int tiles_x = (p.ow + 63) / 64, tiles_y = (p.oh + C::WP - 1) / C::WP;
  const int n_tiles = tiles_x * tiles_y * p.n;
  const int n_cb = (p.cout + 63) / 64;
  // resident workgroups: two per CU (launch bounds), a whole number per output block
  int per_cb = 512 / n_cb;
  if (per_cb < 1) per_cb = 1;
  if (per_cb > n_tiles) per_cb = n_tiles;
  const int grid = per_cb * n_cb;
  const unsigned long long opix = (unsigned long long)p.n * p.yh * p.yw - 1;
  const bool spans_ok = (opix * p.y_ld + p.cout) * 2ull < 0xFFFFFF00ull &&
                        (!p.res || (opix * p.res_ld + p.cout) * 2ull < 0xFFFFFF00ull) &&
                        (!p.dact || (opix * p.z_ld + p.cout) * 2ull < 0xFFFFFF00ull);
  if (p.out_f32)
    DVIE_LAUNCH((conv_nk_kernel<CP8, true>), dim3(grid), dim3(512), 0, s, p, n_cb, n_tiles, tiles_x, tiles_y);
  else if (nk_pre_on() && spans_ok && (p.res || p.beta || p.dact))  // (no operands: the seg encoder's
    // 20 -> 32 forward measured 0.136 -> 0.142 ms with the prefetch form, profiles/r06/nkpre_*)
    DVIE_LAUNCH((conv_nk_kernel<CP8, false, true>), dim3(grid), dim3(512), 0, s, p, n_cb, n_tiles, tiles_x, tiles_y);
  else
    DVIE_LAUNCH((conv_nk_kernel<CP8, false>), dim3(grid), dim3(512), 0, s, p, n_cb, n_tiles, tiles_x, tiles_y);
}

// ---------------------------------------------------------------------------------------
// Eight-row halo tiles (conv_h8_kernel): stride-1 3x3 convs with c % 32 == 0 and
// cout % 128 == 0 -- HRNet's 128- and 256-channel branch convs and their data gradients.
//
// Against conv_halo_kernel<2,2,4,3,3> (4 output rows x 64 px x 128 channels, 64-channel
// chunks, one barrier per tap) this tile is twice as tall at half the chunk depth, so each
// streamed weight byte feeds twice the pixels and the LDS-DMA feed per MFMA drops from
// 24 KB to 14 KB per 16 MFMAs per wave; one tap COLUMN (3 taps, 24 KB of weights) is staged
// per super-step, so the barrier + vmcnt wait come once per 48 MFMAs instead of 16, and the
// weights of the next column get a whole super-step of cover.  A wave owns 64 channels x
// 2 rows x 64 px (8 accumulators); inside a column the three taps shift the halo by one row,
// so a B fragment row is read once per (column, slice) and used by two taps.  The column's
// wait + barrier sit before its last eight MFMAs, which then cover the LDS round trip of the
// next column's first fragments (same box: 256 -> 256 66.9 -> 65.2 us, step 221.2 -> 223.6
// frames/s, profiles/r04h8b/).
//   LDS: halo 10 x 66 px x 80 B (32 channels + 16 B pad: conflict-free b128 reads for any
//   16 consecutive pixels), double buffered (2 x 56 KB); weights 2 x 3 x (128 rows x 64 B,
//   16-B chunks XOR-swizzled by (row >> 2) & 3) = 48 KB.  160 KB total, one workgroup per CU.
//   Epilogue operands (residual / accumulate / activation input: EPI bits 1 / 2 / 4) are
//   compile-time, loaded with buffer loads (out-of-range lanes read zeros, no branches).
struct H8 {
  static constexpr int NW = 8, NTH = 512;
  static constexpr int BC = 128, PR = 8, KC = 32;
  static constexpr int HR = PR + 2, HWD = 66, PITCH = 80;
  static constexpr int HSLOTS = HR * HWD * 5;
  static constexpr int NHI = ((HSLOTS + 63) / 64 + NW - 1) / NW * NW;
  static constexpr int NHQ = NHI / NW;
  static constexpr int HSZ = NHI * 1024;
  static constexpr int ASZ = BC * KC * 2;  // one tap
  static constexpr int WSZ = 3 * ASZ;      // one tap column
  static constexpr int SMEM = 2 * HSZ + 2 * WSZ;
  static constexpr int H0 = 4;             // halo pieces per wave issued in column 0 (rest in column 1)
};
static_assert(H8::SMEM <= 163840, "conv_h8 LDS budget");
static_assert(H8::NHQ == 7 && H8::H0 < H8::NHQ, "halo shares");

template <int EPI>
__global__ __launch_bounds__(512) void conv_h8_kernel(const dvie_conv_desc p, int n_ct, int n_tiles, int tiles_x,
                                                      int tiles_y) {
  typedef H8 C;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave >> 2, wp = wave & 3;
  const int r32 = lane & 31, hh = lane >> 5;
  const int nchunks = p.c >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // persistent: XCD g (= blockIdx % 8) takes a contiguous tile range, its blocks stride it
  const int G = gridDim.x, g = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nbg = G / 8 + (g < G % 8 ? 1 : 0);
  const int q8 = n_tiles / 8, r8 = n_tiles % 8;
  const int ts = g < r8 ? g * (q8 + 1) : r8 * (q8 + 1) + (g - r8) * q8;
  const int tile0 = ts + jb, tile_end = ts + q8 + (g < r8 ? 1 : 0);
  if (tile0 >= tile_end) return;

  auto tile_job = [&](int t) {
    JobInfo J;
    J.t = t;
    J.k = 0;
    J.valid = t < tile_end;
    J.c0 = (t % n_ct) * C::BC;
    int pt = t / n_ct;
    J.x0 = (pt % tiles_x) * 64;
    pt /= tiles_x;
    J.y0 = (pt % tiles_y) * C::PR;
    J.n = pt / tiles_y;
    return J;
  };
  auto next_job = [&](const JobInfo& J) {
    if (J.k + 1 < nchunks) {
      JobInfo N = J;
      N.k = J.k + 1;
      return N;
    }
    return tile_job(J.t + nbg);
  };

  // halo DMA geometry: slot -> (row, column, 16-B channel group; group 4 = pad)
  int hgeo[C::NHQ];
#pragma unroll
  for (int q = 0; q < C::NHQ; ++q) {
    const int slot = (wave + C::NW * q) * 64 + lane;
    const int hr = slot / 5, cs = slot - 5 * (slot / 5);
    const int hy = hr / C::HWD, hx = hr - (hr / C::HWD) * C::HWD;
    hgeo[q] = (cs < 4 && hr < C::HR * C::HWD) ? (hy << 16) | (hx << 4) | cs : -1;
  }
  // weight DMA: lane fills chunk (lane & 3) of row 16*wave + (lane >> 2) from source chunk
  // (lane & 3) ^ ((row >> 2) & 3)
  const int arow = wave * 16 + (lane >> 2);
  const unsigned aoff = (unsigned)arow * (unsigned)p.kpad * 2u + (unsigned)((((lane & 3) ^ ((arow >> 2) & 3))) * 16);
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;

  char* const Hs = smem;
  char* const As = smem + 2 * C::HSZ;

  auto halo_issue = [&](const JobInfo& J, int hb, int qa, int qb) {
    const int nrec = J.valid ? (int)(xbytes - (unsigned long long)J.k * 64) : 0;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + (size_t)J.k * 64), 0, nrec, 0x00020000);
    char* dst = Hs + hb * C::HSZ + wave * 1024;
    const int ybase = J.y0 + p.dy0, xbase = J.x0 + p.dx0;
#pragma unroll
    for (int q = qa; q < qb; ++q) {
      const int gq = hgeo[q];
      const int iy = ybase + (gq >> 16), ix = xbase + ((gq >> 4) & 0xFFF);
      const bool ok = gq >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
      const unsigned o = ok ? (unsigned)((J.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(gq & 15) * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(dst + q * C::NW * 1024), 16, o, 0, 0, 0);
    }
  };
  // tap (ti, v) of job J's tap column v into weight buffer ab (tap index ti*3 + v)
  auto a_issue = [&](const JobInfo& J, int v, int ab, int ti) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, J.valid ? (int)wbytes : 0, 0x00020000);
    const unsigned so = (unsigned)(J.c0 * p.kpad + (ti * 3 + v) * p.c + 32 * J.k) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(As + ab * C::WSZ + ti * C::ASZ + wave * 1024), 16, aoff, so, 0,
                                             0);
  };

  // fragment addresses: A row wc*64 + r32 (+32 i), chunk (2s + hh) swizzled; B pixel r32 of
  // halo row 2*wp (+ tap row + accumulator row), channel group hh of slice s
  const int arw = wc * 64 + r32;
  const int a_s0 = arw * 64 + (((0 + hh) ^ ((arw >> 2) & 3)) << 4);
  const int a_s1 = arw * 64 + (((2 + hh) ^ ((arw >> 2) & 3)) << 4);
  const int b_base = (2 * wp * C::HWD + r32) * C::PITCH + hh * 16;

  f32x16 acc[2][2][2];  // [i: 32-channel block][r: row][b: 32-pixel half]

  {
    const JobInfo J0 = tile_job(tile0);
    halo_issue(J0, 0, 0, C::NHQ);
#pragma unroll
    for (int ti = 0; ti < 3; ++ti) a_issue(J0, 0, 0, ti);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  int hb = 0, ab = 0;
  JobInfo J = tile_job(tile0);
  JobInfo J1 = next_job(J);
  // phase-0 fragments of a column (A: tap row 0, slice 0; B: halo rows 0 and 1, slice 0).
  // They are loaded right after the barrier that ends the previous column, under that
  // column's last eight MFMAs, so no column starts on an LDS round trip.
  i32x4 pa[2], pb[2][2];
  auto load_p0 = [&](const char* A0, const char* H0, int v0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) pa[i] = *(const i32x4*)(A0 + a_s0 + i * 2048);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int b = 0; b < 2; ++b) pb[r][b] = *(const i32x4*)(H0 + (r * C::HWD + 32 * b + v0) * C::PITCH);
  };
  load_p0(As, Hs + b_base, 0);
  while (J.valid) {
    if (J.k == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][r][b][e] = 0.f;
    }
    const char* H = Hs + hb * C::HSZ + b_base;
    const bool tile_end_job = J.k + 1 == nchunks;  // the epilogue follows this job
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const char* A = As + ab * C::WSZ;
      const JobInfo& JW = v < 2 ? J : J1;  // owner of the next column's weights
      const int vw = v < 2 ? v + 1 : 0;
      i32x4 af[2][3][2], bf[2][4][2];
      auto load_a = [&](int s, int ti) {
#pragma unroll
        for (int i = 0; i < 2; ++i) af[s][ti][i] = *(const i32x4*)(A + (s ? a_s1 : a_s0) + ti * C::ASZ + i * 2048);
      };
      auto load_b = [&](int s, int row) {
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[s][row][b] = *(const i32x4*)(H + (row * C::HWD + 32 * b + v) * C::PITCH + s * 32);
      };
#pragma unroll
      for (int i = 0; i < 2; ++i) af[0][0][i] = pa[i];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[0][r][b] = pb[r][b];
#pragma unroll
      for (int ph = 0; ph < 6; ++ph) {
        const int s = ph / 3, ti = ph % 3;
        // fragments of the next phase
        if (ph < 5) {
          const int s2 = (ph + 1) / 3, t2 = (ph + 1) % 3;
          load_a(s2, t2);
          if (t2 == 0) {
            load_b(s2, 0);
            load_b(s2, 1);
          } else {
            load_b(s2, t2 + 1);
          }
        }
        // DMA: the next column's three weight taps first, then this column's halo share
        // (the end-of-column wait counts on the halo pieces being the youngest)
        if (ph < 3) a_issue(JW, vw, ab ^ 1, ph);
        if (v == 0 && ph == 3) halo_issue(J1, hb ^ 1, 0, 2);
        if (v == 0 && ph == 4) halo_issue(J1, hb ^ 1, 2, 3);
        if (v == 0 && ph == 5) halo_issue(J1, hb ^ 1, 3, C::H0);
        if (v == 1 && ph == 3) halo_issue(J1, hb ^ 1, C::H0, C::H0 + 1);
        if (v == 1 && ph == 4) halo_issue(J1, hb ^ 1, C::H0 + 1, C::H0 + 2);
        if (v == 1 && ph == 5) halo_issue(J1, hb ^ 1, C::H0 + 2, C::NHQ);
        if (ph == 5) {
          // end of the column before its last MFMAs: the next column's weights (and, after
          // column 2, the next job's halo) have landed -- this column's halo share may stay
          // in flight -- and every wave's reads of this column's weight buffer are done
          // (lgkmcnt 0), so the buffer may be refilled after the barrier
          if (v == 0)
            DVIE_VMCNT_LGKM0(C::H0);
          else if (v == 1)
            DVIE_VMCNT_LGKM0(C::NHQ - C::H0);
          else
            DVIE_VMCNT_LGKM0(0);
          __builtin_amdgcn_s_barrier();
          if (v < 2)
            load_p0(As + (ab ^ 1) * C::WSZ, H, v + 1);
          else if (!tile_end_job)
            load_p0(As + (ab ^ 1) * C::WSZ, Hs + (hb ^ 1) * C::HSZ + b_base, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[i][r][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[s][ti][i]),
                                                                     __builtin_bit_cast(bf16x8, bf[s][ti + r][b]),
                                                                     acc[i][r][b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      ab ^= 1;
    }
    hb ^= 1;

    if (J.k + 1 == nchunks) {
      // ---- epilogue: eight groups (channel block i, row r, pixel half b), one accumulator each; the
      // operands of group g+1 are issued before the arithmetic of group g ----
      const long long pix0 = ((long long)J.n * p.yh + (long long)J.y0 * p.osy + p.ory) * p.yw + (long long)J.x0 * p.osx + p.orx;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const bf16_t*)p.res + ((EPI & 1) ? pix0 * p.res_ld : 0)), 0, 0x7FFFFFF0, 0x00020000);
      const __amdgpu_buffer_rsrc_t rb =
          __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16_t*)p.y + pix0 * p.y_ld), 0, 0x7FFFFFF0, 0x00020000);
      const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const bf16_t*)p.z + ((EPI & 4) ? pix0 * p.z_ld : 0)), 0, 0x7FFFFFF0, 0x00020000);
      i32x4 o_r[2][2], o_b[2][2], o_z[2][2];  // [buffer][P]
      // group gi: row r = gi >> 2, pixel half b = (gi >> 1) & 1, channel block i = gi & 1
      auto epi_load = [&](int gi) {
        const int i = gi & 1, r = gi >> 2, b = (gi >> 1) & 1, u = gi & 1;
#pragma unroll
          for (int P = 0; P < 2; ++P) {
            const int oy = J.y0 + 2 * wp + r, ox = J.x0 + 32 * b + r32;
            const int co = J.c0 + wc * 64 + 32 * i + 16 * P + 8 * hh;
            const bool ok = oy < p.oh && ox < p.ow;
            const long long dp = (long long)(2 * wp + r) * p.osy * p.yw + (long long)(32 * b + r32) * p.osx;
            if (EPI & 1) o_r[u][P] = __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? (unsigned)((dp * p.res_ld + co) * 2) : OOB, 0, 0);
            if (EPI & 2) o_b[u][P] = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? (unsigned)((dp * p.y_ld + co) * 2) : OOB, 0, 0);
            if (EPI & 4) o_z[u][P] = __builtin_amdgcn_raw_buffer_load_b128(rz, ok ? (unsigned)((dp * p.z_ld + co) * 2) : OOB, 0, 0);
          }
      };
      if (EPI) epi_load(0);
#pragma unroll
      for (int gi = 0; gi < 8; ++gi) {
        const int i = gi & 1, r = gi >> 2, b = (gi >> 1) & 1, u = gi & 1;
        if (EPI && gi < 7) epi_load(gi + 1);
        __builtin_amdgcn_sched_barrier(0);
        {
          float v8[2][8];
#pragma unroll
          for (int P = 0; P < 2; ++P)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][r][b][8 * P + e]),
                                                               __float_as_uint(acc[i][r][b][8 * P + 4 + e]), false, false);
              v8[P][e] = __uint_as_float(sw[0]);
              v8[P][4 + e] = __uint_as_float(sw[1]);
            }
          const int oy = J.y0 + 2 * wp + r, ox = J.x0 + 32 * b + r32;
          const bool ok = oy < p.oh && ox < p.ow;
          const long long dp = (long long)(2 * wp + r) * p.osy * p.yw + (long long)(32 * b + r32) * p.osx;
#pragma unroll
          for (int P = 0; P < 2; ++P) {
            const int co = J.c0 + wc * 64 + 32 * i + 16 * P + 8 * hh;
            float* w = v8[P];
            if (p.bias) {
              const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[e] += b0[e];
                w[4 + e] += b1[e];
              }
            }
            if (EPI & 1) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[2 * e] += __uint_as_float(((uint32_t)o_r[u][P][e]) << 16);
                w[2 * e + 1] += __uint_as_float(((uint32_t)o_r[u][P][e]) & 0xffff0000u);
              }
            }
            if (EPI & 2) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[2 * e] += __uint_as_float(((uint32_t)o_b[u][P][e]) << 16);
                w[2 * e + 1] += __uint_as_float(((uint32_t)o_b[u][P][e]) & 0xffff0000u);
              }
            }
            act_apply(w, 8, p.act, p.alpha);
            if (EPI & 4) {
              float z[8];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                z[2 * e] = __uint_as_float(((uint32_t)o_z[u][P][e]) << 16);
                z[2 * e + 1] = __uint_as_float(((uint32_t)o_z[u][P][e]) & 0xffff0000u);
              }
              dact_apply(w, z, 8, p.dact, p.alpha);
            }
            i32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (int)pack_bf16x2(w[2 * e], w[2 * e + 1]);
            if (ok) __builtin_amdgcn_raw_buffer_store_b128(o, rb, (unsigned)((dp * p.y_ld + co) * 2), 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      load_p0(As + ab * C::WSZ, Hs + hb * C::HSZ + b_base, 0);  // the next job's first column
    }
    J = J1;
    J1 = next_job(J1);
  }
}

// DVIE_CONV_H8=0: the 4-row halo kernel takes these convs (A/B runs); read per launch
static bool h8_on() {
  const char* e = getenv("DVIE_CONV_H8");
  return !(e && *e == '0');
}

template <int EPI>
static void launch_h8(const dvie_conv_desc& p, hipStream_t s, int n_ct, int n_tiles, int tiles_x, int tiles_y) {
  const int grid = n_tiles > 256 ? 256 : n_tiles;
  DVIE_LAUNCH((conv_h8_kernel<EPI>), dim3(grid), dim3(H8::NTH), 0, s, p, n_ct, n_tiles, tiles_x, tiles_y);
}

// 3x3 stride-1 conv, identity taps (t3), bf16 output; true when the eight-row kernel took it
static bool conv_h8_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (!h8_on() || p.out_f32 || p.c % 32 != 0 || p.c < 64 || p.cout % 128 != 0) return false;
  const int n_ct = p.cout / H8::BC, tiles_x = (p.ow + 63) / 64, tiles_y = (p.oh + H8::PR - 1) / H8::PR;
  const long long nt = (long long)n_ct * tiles_x * tiles_y * p.n;
  if (nt < 224 || nt >= (1LL << 30)) return false;  // fewer tiles than CUs: the 4-row kernel
  const int n_tiles = (int)nt;
  switch ((p.res ? 1 : 0) | (p.beta ? 2 : 0) | (p.dact ? 4 : 0)) {
    case 0: launch_h8<0>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 1: launch_h8<1>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 2: launch_h8<2>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 3: launch_h8<3>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 4: launch_h8<4>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 5: launch_h8<5>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    case 6: launch_h8<6>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
    default: launch_h8<7>(p, s, n_ct, n_tiles, tiles_x, tiles_y); break;
  }
  return true;
}

// DVIE_CONV_NK=0: narrow-input 3x3 convs on the chunked kernels (A/B runs)
static const bool nk_env_off = getenv("DVIE_CONV_NK") && *getenv("DVIE_CONV_NK") == '0';

bool conv_narrow_launch(const dvie_conv_desc& p, hipStream_t s);  // conv_narrow.hip

// DVIE_PH4_CFG: tile configuration of the one-launch stride-2 data gradient (3 = 64 channels
// x 4 rows, 4 = 128 x 4; A/B runs)
static int ph4_cfg(const dvie_conv_desc& p) {
  const char* e = getenv("DVIE_PH4_CFG");
  if (e && *e) return atoi(e);
  return p.cout % 128 == 0 ? 4 : 3;
}

// The stride-2 data gradient's four phases in one launch (dvie_conv_desc.phc > 0); false:
// the descriptor does not meet the kernel's conditions (the caller reports it).
bool conv_halo_ph4_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (p.dtype != DVIE_BF16 || p.out_f32 || p.bias || p.phc <= 0 || p.phc % 32 != 0 || p.cout != 4 * p.phc) return false;
  if (p.th != 2 || p.tw != 2 || p.dy0 != 0 || p.dx0 != 0 || p.ddy != 1 || p.ddx != 1 || p.sy != 1 || p.sx != 1)
    return false;
  if (p.osy != 2 || p.osx != 2 || p.ory != 0 || p.orx != 0) return false;
  if (p.c % 64 != 0 && p.c > 64) return false;
  const unsigned long long pix = (unsigned long long)p.n * p.ih * p.iw;
  if (pix >= (1ull << 31) || ((pix - 1) * (unsigned long long)p.x_ld + (unsigned long long)p.c) * 2ull >= 0xFFFFFF00ull)
    return false;
  return ph4_cfg(p) == 3 ? try_halo<1, 2, 4, 2, 2, true>(p, s) : try_halo<2, 2, 4, 2, 2, true>(p, s);
}

// Returns true when the halo kernel took the launch.
bool conv_halo_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (p.dtype != DVIE_BF16) return false;
  if (p.sy != 1 || p.sx != 1 || p.ddy != 1 || p.ddx != 1) return false;
  if (p.osy < 1 || p.osx < 1 || p.ory < 0 || p.orx < 0) return false;
  if (p.c % 64 != 0 && p.c > 64) return false;  // (c < 64: channels padded with zeros)
  const bool t1 = p.th == 1 && p.tw == 1, t3 = p.th == 3 && p.tw == 3;
  const bool t22 = p.th == 2 && p.tw == 2, t12 = p.th == 1 && p.tw == 2, t21 = p.th == 2 && p.tw == 1;
  if (!t1 && !t3 && !t22 && !t12 && !t21) return false;
  const unsigned long long pix = (unsigned long long)p.n * p.ih * p.iw;
  if (pix >= (1ull << 31)) return false;
  // 32-bit halo offsets: the input's byte span must fit (dvie_conv2d_fwd rejects larger
  // inputs for every kernel; kept here so the halo path never relies on the caller)
  if (((pix - 1) * (unsigned long long)p.x_ld + (unsigned long long)p.c) * 2ull >= 0xFFFFFF00ull) return false;
  int cfg = env_cfg();
  if (cfg == -1) return false;
  if (t3 && !nk_env_off && cfg == -3 && p.c % 8 == 0 && p.c <= 24 && p.kpad >= 9 * p.c) {
    switch (p.c / 8) {
      case 1: launch_nk<1>(p, s); break;
      case 2: launch_nk<2>(p, s); break;
      default: launch_nk<3>(p, s); break;
    }
    return true;
  }
  if (t3 && p.c <= 64 && p.cout <= 64 && (cfg == -3 || cfg == 8) && (long long)p.n * p.oh * p.ow >= 65536) {
    // single input chunk, one 64-channel output tile: weights stay in VGPRs
    switch ((p.c + 15) / 16) {
      case 1: if (!launch_strip<1>(p, s)) launch_ws<1>(p, s); break;
      case 2: if (!launch_strip<2>(p, s)) launch_ws<2>(p, s); break;
      case 3: if (!launch_strip<3>(p, s)) launch_ws<3>(p, s); break;
      default: if (!launch_strip<4>(p, s)) launch_ws<4>(p, s); break;
    }
    return true;
  }
  // <= 32 output channels from > 64 input channels (the HRNet heads): one step per 32-channel
  // chunk with all 9 taps (conv_narrow.hip)
  if (t3 && cfg == -3 && conv_narrow_launch(p, s)) return true;
  if (t3 && cfg == -3 && conv_h8_launch(p, s)) return true;
  if (cfg < 0) {  // measured on MI355X (tools/conv_tune.py): see DESIGN.md
    if (p.cout <= 32)
      cfg = 2;
    else if (t1)  // 1x1: wide weight tiles amortise the per-chunk pixel tile
      cfg = p.cout <= 64 ? 3 : (p.c <= 64 ? 5 : 4);
    else
      cfg = (p.cout <= 64 || p.cout % 128 != 0) ? 3 : 4;
    // fewer 4-row tiles than CUs (VGG19's deep data gradients on 8 frames, 512 -> 512 at
    // 16 x 32 and 512 -> 256 at 32 x 64): 2-row tiles of the same 128 channels fill the chip,
    // 52.9 -> 40.9 and 55.5 -> 43.5 us (profiles/r06/vgg_tune.txt)
    if (t3 && cfg == 4 && (long long)(p.cout / 128) * ((p.ow + 63) / 64) * ((p.oh + 3) / 4) * p.n < 256) cfg = 5;
  }
  if (t3) return launch_cfg<3, 3>(cfg, p, s);
  if (t1) return launch_cfg<1, 1>(cfg, p, s);
  // stride-2 data-gradient phases: two configurations only
  const int c2 = p.cout <= 64 || p.cout % 128 != 0 ? 3 : 4;
  if (t22) return launch_cfg2<2, 2>(c2, p, s);
  if (t12) return launch_cfg2<1, 2>(c2, p, s);
  return launch_cfg2<2, 1>(c2, p, s);
}

}  // namespace dvie
