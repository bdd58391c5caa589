// 1x1 convolution as a plain GEMM for gfx950, bf16: out[pix][co] = sum_ci x[pix][ci] * w[co][ci]
// (forward 1x1 convs of HRNet's bottlenecks / fuse layers, and the data gradient of 1x1 convs,
// including the 1x1 stride phases of strided data gradients through the output placement).
//
// A 1x1 conv needs no spatial tiling: a workgroup owns BP consecutive pixels and BC output
// channels (448-channel layers take two 256-channel column tiles) and walks the input
// channels in K-steps of KC channels.  Both operands are staged by LDS-DMA into XOR-swizzled
// rows (x tile BP x 2KC bytes, weight tile BC x 2KC bytes), NS stages in the ring.  The
// waves form an NWP x NWC grid; each owns 32*MI pixels x 32*TMC channels (MI*TMC
// accumulators of 32x32): per 16-deep k-slice it reads MI pixel fragments and TMC weight
// fragments from LDS and issues MI*TMC MFMAs (v_mfma_f32_32x32x16_bf16).  LDS reads bound
// the wide layers, so the 64-pixel x 128-channel wave tile (6 fragments per 8 MFMAs) beats
// the 32 x 224 one (8 per 7) even though it pads 448 channels to 512.  Epilogue from registers (permlane32 pairing to 16-byte rows)
// with bias / residual / accumulate / activation / activation-derivative fused.
//
// Reference op replaced: nn.Conv2d(kernel_size=1) forward and backward-data (nets/HRNet.py
// bottleneck conv1/conv3, downsample, fuse and final layers).
#include <stdlib.h>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_1x1;

#define DVIE_VMCNT1(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4) | (15 << 8))

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

__device__ __forceinline__ void act1(float* v, int act, float alpha) {
  if (act == DVIE_ACT_LRELU) {
    for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : v[k] * alpha;
  } else if (act == DVIE_ACT_RELU) {
    for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
  } else if (act == DVIE_ACT_ELU) {
    for (int k = 0; k < 8; ++k) v[k] = elu_bf(v[k]);  // (bf16-input kernels: common.h)
  } else if (act == DVIE_ACT_TANH) {
    for (int k = 0; k < 8; ++k) v[k] = tanh_bf(v[k]);
  }
}

__device__ __forceinline__ void dact1(float* v, const float* z, int dact, float alpha) {
  if (dact == DVIE_ACT_LRELU) {
    for (int k = 0; k < 8; ++k) v[k] *= z[k] > 0.f ? 1.f : alpha;
  } else if (dact == DVIE_ACT_RELU) {
    for (int k = 0; k < 8; ++k) v[k] = z[k] > 0.f ? v[k] : 0.f;
  } else if (dact == DVIE_ACT_ELU) {
    for (int k = 0; k < 8; ++k) v[k] *= z[k] > 0.f ? 1.f : z[k] + 1.f;
  } else if (dact == DVIE_ACT_TANH) {
    for (int k = 0; k < 8; ++k) v[k] *= 1.f - z[k] * z[k];
  }
}

__device__ __forceinline__ void unpack8(const i32x4 t, float* v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(((uint32_t)t[e]) << 16);
    v[2 * e + 1] = __uint_as_float(((uint32_t)t[e]) & 0xffff0000u);
  }
}

// 8 x 8 transpose of 16-B chunks inside each 8-lane group: (lane b, chunk k) <-> (lane k,
// chunk b); at distance d the lane with bit d set trades its chunk k for the partner's chunk
// k + d.  An involution: applied to chunks loaded in the transposed (row-coalesced) layout it
// yields the MFMA layout, applied to MFMA-layout results it yields whole-row stores.
// (element-wise selects on the lane bit, so every array index is a constant and the chunks
// stay in registers)
__device__ __forceinline__ void transpose8x8(i32x4 (&ob)[8], int lane) {
  const int b = lane & 7;
#pragma unroll
  for (int d = 4; d >= 1; d >>= 1) {
    const bool up = (b & d) != 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k & d) continue;
      i32x4 t, r;
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = up ? ob[k][e] : ob[k + d][e];
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = __shfl_xor(t[e], d);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ob[k][e] = up ? r[e] : ob[k][e];
        ob[k + d][e] = up ? ob[k + d][e] : r[e];
      }
    }
  }
}

// KC = input channels per K-step (64: 128-byte LDS rows, 32: 64-byte rows, half the stage
// bytes, so the same LDS holds twice the stages in flight).  A DMA piece is always 1 KB:
// RPP rows of RB bytes.
// Wave grid: NWP x NWC waves; a wave owns 32*MI pixels x 32*TMC channels (MI*TMC
// accumulators of 32x32), so per 16-deep k-slice it reads MI + TMC fragments for MI*TMC MFMAs.
template <int TMC, int NS, int KC, int NWP, int MI = 1, int NWC = 1>
struct G1Cfg {
  static constexpr int NW = NWP * NWC;
  static constexpr int BC = 32 * TMC * NWC;
  static constexpr int BP = 32 * MI * NWP;
  static constexpr int RB = KC * 2;              // LDS row bytes
  static constexpr int NCH = RB / 16;            // 16-byte chunks per row (8 or 4)
  static constexpr int RPP = 64 / NCH;           // rows per 1 KB piece (8 or 16)
  static constexpr int NSL = KC / 16;            // 16-deep MFMA k-slices per K-step
  static constexpr int XSZ = BP * RB;
  static constexpr int WSZ = BC * RB;
  static constexpr int STAGE = XSZ + WSZ;
  static constexpr int SMEM = NS * STAGE;  // NS stages: NS-1 K-steps in flight
  static constexpr int XQ = BP / RPP / NW;            // x pieces per wave
  static constexpr int WQ = (BC / RPP + NW - 1) / NW;  // weight pieces per wave (upper bound)
  // chunk swizzle: the 16 rows one ds_read_b128 pass touches land on distinct banks
  static __device__ __forceinline__ int swz(int row) { return NCH == 8 ? (row >> 1) & 7 : (row >> 2) & 3; }
};

// PRE (bf16 output, single K-step only): epilogue operands loaded into registers right after
// the stage's DMA, so their HBM latency overlaps the operand DMA instead of following the
// MFMAs (1 residual, 2 accumulate target, 4 activation input).
// CE (bf16 output, MI = 1, 8 accumulator chunks per lane, identity placement, full channel
// tiles): the packed outputs are transposed across each 8-lane group (three xor-shuffle
// stages), so store instruction k writes 4 whole pixels x 256 B instead of 32 pixels x 32 B.
template <int TMC, int NS, int KC, int NWP, int MI, int NWC, bool OUTF32, int PRE = 0, bool CE = false>
__global__ __launch_bounds__(64 * NWP * NWC) void conv1x1_kernel(const dvie_conv_desc p, int n_ct, int n_tiles, int dbg) {
  dbg = DVIE_DBG(dbg);
  typedef G1Cfg<TMC, NS, KC, NWP, MI, NWC> C;
  constexpr int NW = C::NW;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // tile: co tile fastest (consecutive workgroups share the pixel tile in L2), XCD-contiguous
  const int g = blockIdx.x & 7, i8 = blockIdx.x >> 3;
  const int q8 = n_tiles >> 3, r8 = n_tiles & 7;
  const int bid = (g < r8 ? g * (q8 + 1) : r8 * (q8 + 1) + (g - r8) * q8) + i8;
  const int c0 = (bid % n_ct) * C::BC;
  const int p0 = (bid / n_ct) * C::BP;
  const int npix = p.n * p.oh * p.ow;
  const int nk = (p.c + KC - 1) / KC;

  // DMA lane geometry: piece = RPP rows x RB bytes; lane -> row RPP*piece + lane / NCH, LDS
  // chunk (lane % NCH) holding source chunk (lane % NCH) ^ swz(row)
  const int lrow = lane / C::NCH, lch = lane % C::NCH;
  unsigned xo[C::XQ];
#pragma unroll
  for (int q = 0; q < C::XQ; ++q) {
    const int row = (wave + NW * q) * C::RPP + lrow;
    const int cs = lch ^ C::swz(row);
    xo[q] = (p0 + row < npix) ? (unsigned)(p0 + row) * (unsigned)p.x_ld * 2u + cs * 16u : OOB;
    if (cs * 8 >= p.c) xo[q] = OOB;  // (c < 64: channel padding)
  }
  unsigned wo[C::WQ];
#pragma unroll
  for (int q = 0; q < C::WQ; ++q) {
    const int row = (wave + NW * q) * C::RPP + lrow;
    const int cs = lch ^ C::swz(row);
    wo[q] = (row < C::BC && cs * 8 < p.c) ? (unsigned)row * (unsigned)p.kpad * 2u + cs * 16u : OOB;
  }
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;

  auto stage = [&](int k, int sb) {
    char* X = smem + sb * C::STAGE;
    char* W = X + C::XSZ;
    // K-step k: channels KC*k .. KC*k+KC-1 (chunks past c land as zeros: range check below)
    const int xr = (int)(xbytes - (unsigned long long)k * C::RB);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + (size_t)k * C::RB), 0, xr, 0x00020000);
    const unsigned wb = (unsigned)(c0 * p.kpad + KC * k) * 2u;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.w + wb), 0, (int)(wbytes - wb), 0x00020000);
    const int cvalid = p.c - KC * k;  // channels of this K-step that exist
#pragma unroll
    for (int q = 0; q < C::XQ; ++q) {
      const int row = (wave + NW * q) * C::RPP + lrow;
      const int cs = lch ^ C::swz(row);
      const unsigned o = cs * 8 < cvalid ? xo[q] : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_1x1)(X + (wave + NW * q) * 1024), 16, o, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < C::WQ; ++q) {
      if (wave + NW * q < C::BC / C::RPP) {
        const int row = (wave + NW * q) * C::RPP + lrow;
        const int cs = lch ^ C::swz(row);
        const unsigned o = cs * 8 < cvalid ? wo[q] : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_1x1)(W + (wave + NW * q) * 1024), 16, o, 0, 0, 0);
      }
    }
  };

  // fragment addresses: pixel rows wp*32*MI + 32*i + r32 (B operand), weight rows
  // wc*32*TMC + 32*j + r32 (A); k-slice s uses chunk 2s + h (32-row offsets keep the swizzle)
  const int wp = wave % NWP, wc = wave / NWP;
  int xf[C::NSL], wf[C::NSL];
#pragma unroll
  for (int s = 0; s < C::NSL; ++s) {
    const int prow = wp * 32 * MI + r32;
    xf[s] = prow * C::RB + (((2 * s + hh) ^ C::swz(prow)) << 4);
    wf[s] = (wc * 32 * TMC + r32) * C::RB + (((2 * s + hh) ^ C::swz(r32)) << 4);
  }

  f32x16 acc[MI][TMC];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < TMC; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // prologue: K-steps 0 .. NS-2 in flight
#pragma unroll
  for (int k = 0; k < (NS > 1 ? NS - 1 : 1); ++k)
    if (k < nk) stage(k, k);

  // epilogue-operand prefetch (PRE): lane (pixel wp*32*MI + 32*i + r32, channels
  // c0 + wc*32*TMC + 32*j + 16*P + 8*h .. +7); identity output placement only (checked at launch)
  static_assert(PRE == 0 || (NS == 1 && !OUTF32), "operand prefetch: single K-step, bf16 output");
  i32x4 pr_r[(PRE & 1) ? MI : 1][TMC][2], pr_b[(PRE & 2) ? MI : 1][TMC][2], pr_z[(PRE & 4) ? MI : 1][TMC][2];
  // CE tiles with two or more operands (layer1's 256-channel data gradients: residual +
  // activation input) load them row-coalesced: 0.47 -> 0.43 ms each; with a single operand
  // the transposes' extra registers cost an occupancy step (121 -> 148 VGPRs) and the
  // forward with a residual measured 0.247 -> 0.290 ms (profiles/r05l/)
  constexpr bool CEL = CE && (PRE & (PRE - 1)) != 0;
  if constexpr (CEL) {
    // CE tiles: the operands are loaded in the transposed layout of the CE stores -- lane
    // (h, 8 a + b), chunk k = pixel 8 a + k, channels 16 b + 8 h of the wave's 128 -- so each
    // load instruction reads 4 pixels x 256 contiguous bytes; transpose8x8 (epilogue) turns
    // them into the MFMA layout.  (CE: MI = 1, 8 chunks, full channel tiles.)
    const int wp0 = wave % NWP, wc0 = wave / NWP;
    const int a8 = r32 >> 3, bl = lane & 7;
    const int co = c0 + wc0 * 32 * TMC + 16 * bl + 8 * hh;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int pix = p0 + wp0 * 32 + 8 * a8 + k;
      const bool ok = pix < npix;
      const long long q = ok ? pix : 0;
      if constexpr ((PRE & 1) != 0)
        pr_r[0][k >> 1][k & 1] = ok ? *(const i32x4*)((const bf16_t*)p.res + q * p.res_ld + co) : i32x4{0, 0, 0, 0};
      if constexpr ((PRE & 2) != 0)
        pr_b[0][k >> 1][k & 1] = ok ? *(const i32x4*)((const bf16_t*)p.y + q * p.y_ld + co) : i32x4{0, 0, 0, 0};
      if constexpr ((PRE & 4) != 0)
        pr_z[0][k >> 1][k & 1] = ok ? *(const i32x4*)((const bf16_t*)p.z + q * p.z_ld + co) : i32x4{0, 0, 0, 0};
    }
  } else if constexpr (PRE != 0) {
    const int wp0 = wave % NWP, wc0 = wave / NWP;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < TMC; ++j)
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          const int pix = p0 + wp0 * 32 * MI + 32 * i + r32;
          const int co = c0 + wc0 * 32 * TMC + 32 * j + 16 * P + 8 * hh;
          const bool ok = pix < npix && co < p.cout;
          const long long q = ok ? pix : 0;
          if constexpr ((PRE & 1) != 0)
            pr_r[i][j][P] = ok ? *(const i32x4*)((const bf16_t*)p.res + q * p.res_ld + co) : i32x4{0, 0, 0, 0};
          if constexpr ((PRE & 2) != 0)
            pr_b[i][j][P] = ok ? *(const i32x4*)((const bf16_t*)p.y + q * p.y_ld + co) : i32x4{0, 0, 0, 0};
          if constexpr ((PRE & 4) != 0)
            pr_z[i][j][P] = ok ? *(const i32x4*)((const bf16_t*)p.z + q * p.z_ld + co) : i32x4{0, 0, 0, 0};
        }
  }
  for (int k = 0; k < nk; ++k) {
    const int sb = k % NS;
    // stage k has landed for every wave: this wave's own pieces by the counted wait (stage
    // k+1, issued after it, may stay in flight), the other waves' by the barrier
    if constexpr (NS >= 3) {
      // stages k+1 .. k+NS-2 were issued after stage k: that many may stay in flight
      static_assert(NS <= 5, "wait table covers up to 3 stages in flight");
      constexpr int P_HI = C::XQ + C::WQ, P_LO = C::XQ + C::WQ - 1;  // pieces per wave per stage
      static_assert(3 * P_HI < 64, "vmcnt is 6 bits");
      const bool hi = wave + NW * (C::WQ - 1) < C::BC / C::RPP;
      const int m = min(NS - 2, nk - 1 - k);
      if (m >= 3) {
        if (hi) DVIE_VMCNT1(3 * P_HI); else DVIE_VMCNT1(3 * P_LO);
      } else if (m == 2) {
        if (hi) DVIE_VMCNT1(2 * P_HI); else DVIE_VMCNT1(2 * P_LO);
      } else if (m == 1) {
        if (hi) DVIE_VMCNT1(P_HI); else DVIE_VMCNT1(P_LO);
      } else {
        __builtin_amdgcn_s_waitcnt(0);
      }
    } else {
      __builtin_amdgcn_s_waitcnt(0);
    }
    __builtin_amdgcn_s_barrier();
    if (NS > 1 && k + NS - 1 < nk) stage(k + NS - 1, (k + NS - 1) % NS);
    const char* X = smem + sb * C::STAGE;
    const char* W = X + C::XSZ;
    if (dbg & 2) continue;
#pragma unroll
    for (int s = 0; s < C::NSL; ++s) {
      i32x4 b[MI], a[TMC];
#pragma unroll
      for (int i = 0; i < MI; ++i) b[i] = *(const i32x4*)(X + xf[s] + i * 32 * C::RB);
#pragma unroll
      for (int j = 0; j < TMC; ++j) a[j] = *(const i32x4*)(W + wf[s] + j * 32 * C::RB);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < TMC; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[j]),
                                                              __builtin_bit_cast(bf16x8, b[i]), acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: lane owns pixel wp*32*MI + 32*i + r32; after permlane32 pairing, lane half h
  // holds channels 16P + 8h .. +7 of pair P of each 32-channel accumulator
  static_assert(!CE || (MI == 1 && 2 * TMC == 8 && !OUTF32), "coalesced epilogue: 8 chunks per lane");
  if constexpr (CEL) {  // the row-coalesced operand loads into the MFMA layout
    auto tr = [&](i32x4 (&a)[TMC][2]) {
      i32x4 t8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t8[k] = a[k >> 1][k & 1];
      transpose8x8(t8, lane);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k >> 1][k & 1] = t8[k];
    };
    if constexpr ((PRE & 1) != 0) tr(pr_r[0]);
    if constexpr ((PRE & 2) != 0) tr(pr_b[0]);
    if constexpr ((PRE & 4) != 0) tr(pr_z[0]);
  }
  i32x4 ob[CE ? 8 : 1];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
  const int pix0 = p0 + wp * 32 * MI + 32 * i + r32;
  const int pix = CE ? min(pix0, npix - 1) : pix0;  // (CE: every lane takes part in the shuffles)
  float v[TMC][2][8];
#pragma unroll
  for (int j = 0; j < TMC; ++j)
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * P + e]),
                                                         __float_as_uint(acc[i][j][8 * P + 4 + e]), false, false);
        v[j][P][e] = __uint_as_float(sw[0]);
        v[j][P][4 + e] = __uint_as_float(sw[1]);
      }
  if (!CE && pix >= npix) continue;
  long long yp = pix;
  if (p.osy != 1 || p.osx != 1 || p.ory != 0 || p.orx != 0 || p.yh != p.oh || p.yw != p.ow) {
    const int hw = p.oh * p.ow;
    const int n = pix / hw, r = pix - n * hw;
    const int oy = r / p.ow, ox = r - oy * p.ow;
    yp = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
  }
#pragma unroll
  for (int j = 0; j < TMC; ++j)
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      const int co = c0 + wc * 32 * TMC + 32 * j + 16 * P + 8 * hh;
      if (!CE && co >= p.cout) continue;
      float* w = v[j][P];
      if (p.bias) {
        const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[e] += b0[e];
          w[4 + e] += b1[e];
        }
      }
      if constexpr (OUTF32) {
        float* dst = (float*)p.y + yp * p.y_ld + co;
        if (p.res) {
          const float* rs = (const float*)p.res + yp * p.res_ld + co;
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
        for (int k = 0; k < 8; ++k) w[k] = act_f32(w[k], p.act, p.alpha);
        if (p.dact) {
          float z[8];
          unpack8(*(const i32x4*)((const bf16_t*)p.z + yp * p.z_ld + co), z);
          dact1(w, z, p.dact, p.alpha);
        }
        *(f32x4*)dst = f32x4{w[0], w[1], w[2], w[3]};
        *(f32x4*)(dst + 4) = f32x4{w[4], w[5], w[6], w[7]};
      } else {
        bf16_t* dst = (bf16_t*)p.y + yp * p.y_ld + co;
        float t[8];
        if (p.res) {
          if constexpr ((PRE & 1) != 0)
            unpack8(pr_r[(PRE & 1) ? i : 0][j][P], t);
          else
            unpack8(*(const i32x4*)((const bf16_t*)p.res + yp * p.res_ld + co), t);
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] += t[e];
        }
        if (p.beta) {
          if constexpr ((PRE & 2) != 0)
            unpack8(pr_b[(PRE & 2) ? i : 0][j][P], t);
          else
            unpack8(*(const i32x4*)dst, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] += t[e];
        }
        act1(w, p.act, p.alpha);
        if (p.dact) {
          if constexpr ((PRE & 4) != 0)
            unpack8(pr_z[(PRE & 4) ? i : 0][j][P], t);
          else
            unpack8(*(const i32x4*)((const bf16_t*)p.z + yp * p.z_ld + co), t);
          dact1(w, t, p.dact, p.alpha);
        }
        i32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (int)pk_bf16(w[2 * e], w[2 * e + 1]);
        if constexpr (CE)
          ob[2 * j + P] = o;
        else if (!(dbg & 1) || w[0] == 12345.678f)
          *(i32x4*)dst = o;
      }
    }
  }
  if constexpr (CE) {
    transpose8x8(ob, lane);
    const int b = lane & 7;
    // lane (h, 8a + b) now holds pixel 8a + k, channels 32 (b / 2) + 16 (b % 2) + 8 h of chunk k
    const int a8 = r32 >> 3;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int px = p0 + wp * 32 + 8 * a8 + k;
      const int co = c0 + wc * 32 * TMC + 32 * (b >> 1) + 16 * (b & 1) + 8 * hh;
      if (px < npix) *(i32x4*)((bf16_t*)p.y + (long long)px * p.y_ld + co) = ob[k];
    }
  }
}

// Persistent form for multi-K-step layers (bf16 output): a workgroup walks tiles T = b,
// b + G, ... (b its XCD-contiguous id) and the stage ring runs across tile boundaries, so the
// first K-steps of the next tile are in flight while this tile finishes its MFMAs and its
// epilogue (the one-tile-per-workgroup form pays a stage latency at every tile start).
template <int TMC, int NS, int KC, int NWP, int MI, int NWC>
__global__ __launch_bounds__(64 * NWP * NWC) void conv1x1_persist_kernel(const dvie_conv_desc p, int n_ct, int n_tiles) {
  typedef G1Cfg<TMC, NS, KC, NWP, MI, NWC> C;
  constexpr int NW = C::NW;
  static_assert(NS >= 2, "stage ring");
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  const int G = gridDim.x;
  const int g = blockIdx.x & 7, i8 = blockIdx.x >> 3;
  const int q8 = G >> 3, r8 = G & 7;
  const int b = (g < r8 ? g * (q8 + 1) : r8 * (q8 + 1) + (g - r8) * q8) + i8;
  const int npix = p.n * p.oh * p.ow;
  const int nk = (p.c + KC - 1) / KC;
  const int my_tiles = b < n_tiles ? (n_tiles - 1 - b) / G + 1 : 0;
  const int njobs = my_tiles * nk;
  if (njobs == 0) return;

  const int lrow = lane / C::NCH, lch = lane % C::NCH;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;

  // job jj = (tile i = jj / nk of this workgroup, K-step k = jj % nk) into stage sb
  auto stage = [&](int jj, int sb) {
    const int i = jj / nk, k = jj - nk * (jj / nk);
    const int T = b + i * G;
    const int c0 = (T % n_ct) * C::BC, p0 = (T / n_ct) * C::BP;
    char* X = smem + sb * C::STAGE;
    char* W = X + C::XSZ;
    const int xr = (int)(xbytes - (unsigned long long)k * C::RB);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + (size_t)k * C::RB), 0, xr, 0x00020000);
    const unsigned wb = (unsigned)(c0 * p.kpad + KC * k) * 2u;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.w + wb), 0, (int)(wbytes - wb), 0x00020000);
    const int cvalid = p.c - KC * k;
#pragma unroll
    for (int q = 0; q < C::XQ; ++q) {
      const int row = (wave + NW * q) * C::RPP + lrow;
      const int cs = lch ^ C::swz(row);
      const unsigned o = (cs * 8 < cvalid && p0 + row < npix) ? (unsigned)(p0 + row) * (unsigned)p.x_ld * 2u + cs * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_1x1)(X + (wave + NW * q) * 1024), 16, o, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < C::WQ; ++q) {
      if (wave + NW * q < C::BC / C::RPP) {
        const int row = (wave + NW * q) * C::RPP + lrow;
        const int cs = lch ^ C::swz(row);
        const unsigned o = (row < C::BC && cs * 8 < cvalid) ? (unsigned)row * (unsigned)p.kpad * 2u + cs * 16u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_1x1)(W + (wave + NW * q) * 1024), 16, o, 0, 0, 0);
      }
    }
  };

  const int wp = wave % NWP, wc = wave / NWP;
  int xf[C::NSL], wf[C::NSL];
#pragma unroll
  for (int sl = 0; sl < C::NSL; ++sl) {
    const int prow = wp * 32 * MI + r32;
    xf[sl] = prow * C::RB + (((2 * sl + hh) ^ C::swz(prow)) << 4);
    wf[sl] = (wc * 32 * TMC + r32) * C::RB + (((2 * sl + hh) ^ C::swz(r32)) << 4);
  }

  // leave the stages issued after job j (at most NS-2, fewer at the end) in flight
  constexpr int P_HI = C::XQ + C::WQ, P_LO = C::XQ + C::WQ - 1;  // pieces per wave per stage
  static_assert((NS - 2) * P_HI < 64, "vmcnt is 6 bits");
  const bool hi = wave + NW * (C::WQ - 1) < C::BC / C::RPP;
  auto wait_stages = [&](int j) {
    const int m = min(NS - 2, njobs - 1 - j);
    if (m >= 3) {
      if (hi) DVIE_VMCNT1(3 * P_HI); else DVIE_VMCNT1(3 * P_LO);
    } else if (m == 2) {
      if (hi) DVIE_VMCNT1(2 * P_HI); else DVIE_VMCNT1(2 * P_LO);
    } else if (m == 1) {
      if (hi) DVIE_VMCNT1(P_HI); else DVIE_VMCNT1(P_LO);
    } else {
      __builtin_amdgcn_s_waitcnt(0);
    }
  };

  f32x16 acc[MI][TMC];
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (k < njobs) stage(k, k);
  for (int jj = 0; jj < njobs; ++jj) {
    const int k = jj - nk * (jj / nk);
    if (k == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < TMC; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    }
    // job jj landed: this wave's pieces by a counted wait (stages issued after it may stay in
    // flight), other waves' by the barrier.  After an epilogue the wait was done before its
    // stores (so that they never have to drain here).
    if (k != 0 || jj == 0) wait_stages(jj);
    __builtin_amdgcn_s_barrier();
    if (jj + NS - 1 < njobs) stage(jj + NS - 1, (jj + NS - 1) % NS);
    const char* X = smem + (jj % NS) * C::STAGE;
    const char* W = X + C::XSZ;
#pragma unroll
    for (int sl = 0; sl < C::NSL; ++sl) {
      i32x4 bq[MI], a[TMC];
#pragma unroll
      for (int i = 0; i < MI; ++i) bq[i] = *(const i32x4*)(X + xf[sl] + i * 32 * C::RB);
#pragma unroll
      for (int j = 0; j < TMC; ++j) a[j] = *(const i32x4*)(W + wf[sl] + j * 32 * C::RB);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < TMC; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[j]),
                                                              __builtin_bit_cast(bf16x8, bq[i]), acc[i][j], 0, 0, 0);
    }
    if (k + 1 < nk) continue;
    if (jj + 1 < njobs) wait_stages(jj + 1);

    // ---- epilogue of tile T (as conv1x1_kernel, bf16 output)
    const int T = b + (jj / nk) * G;
    const int c0 = (T % n_ct) * C::BC, p0 = (T / n_ct) * C::BP;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int pix = p0 + wp * 32 * MI + 32 * i + r32;
      float v[TMC][2][8];
#pragma unroll
      for (int j = 0; j < TMC; ++j)
#pragma unroll
        for (int P = 0; P < 2; ++P)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * P + e]),
                                                             __float_as_uint(acc[i][j][8 * P + 4 + e]), false, false);
            v[j][P][e] = __uint_as_float(sw[0]);
            v[j][P][4 + e] = __uint_as_float(sw[1]);
          }
      if (pix >= npix) continue;
      long long yp = pix;
      if (p.osy != 1 || p.osx != 1 || p.ory != 0 || p.orx != 0 || p.yh != p.oh || p.yw != p.ow) {
        const int hw = p.oh * p.ow;
        const int n = pix / hw, r = pix - n * hw;
        const int oy = r / p.ow, ox = r - oy * p.ow;
        yp = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
      }
#pragma unroll
      for (int j = 0; j < TMC; ++j)
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          const int co = c0 + wc * 32 * TMC + 32 * j + 16 * P + 8 * hh;
          if (co >= p.cout) continue;
          float* w = v[j][P];
          if (p.bias) {
            const f32x4 b0 = *(const f32x4*)(p.bias + co), b1 = *(const f32x4*)(p.bias + co + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[e] += b0[e];
              w[4 + e] += b1[e];
            }
          }
          bf16_t* dst = (bf16_t*)p.y + yp * p.y_ld + co;
          float t[8];
          if (p.res) {
            unpack8(*(const i32x4*)((const bf16_t*)p.res + yp * p.res_ld + co), t);
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] += t[e];
          }
          if (p.beta) {
            unpack8(*(const i32x4*)dst, t);
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] += t[e];
          }
          act1(w, p.act, p.alpha);
          if (p.dact) {
            unpack8(*(const i32x4*)((const bf16_t*)p.z + yp * p.z_ld + co), t);
            dact1(w, t, p.dact, p.alpha);
          }
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (int)pk_bf16(w[2 * e], w[2 * e + 1]);
          *(i32x4*)dst = o;
        }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// Ring form for the wide multi-K-step layers without epilogue operands (the heads' 448 -> 896
// forward): 256 x 256 tiles, 64-channel K-steps, persistent over the workgroup's tiles.  The
// LDS is a ring of five 32-KB slots, each holding ONE operand of one K-step (the x rows or the
// weight rows, 128-B rows as above); "half-stage" h = operand h & 1 of job h >> 1 (job = tile,
// K-step) lives in slot h % 5.  At job j the slots of job j - 1 are refilled with half-stages
// 2j + 3 and 2j + 4, so three half-stages (96 KB) are in flight after the issue and one at the
// wait -- against the two-stage form's one 64-KB stage, issued in one burst and drained at
// every K-step.  Each wave issues 4 pieces per half-stage (uniform, so the waits are counted).
// The bias is loaded into the accumulators when a tile starts (before that job's DMA issue, so
// waiting for it drains nothing); the epilogue (activation, bf16 stores, general output
// placement) reads no memory.
// AB: timing-only ablations (instantiated in -DDVIE_TIMING_DBG builds only; DVIE_1X1_DBG):
// 1 no stores, 2 no MFMAs, 4 no DMA after the prologue
template <int TMC, int NWP, int MI, int NWC, int ACT, int AB = 0>
__global__ __launch_bounds__(64 * NWP * NWC) void conv1x1_ring_kernel(const dvie_conv_desc p, int n_ct, int n_tiles) {
  constexpr int dbg = AB;
  typedef G1Cfg<TMC, 2, 64, NWP, MI, NWC> C;
  constexpr int NW = C::NW, SL = 32768, NSLOT = 5, PPH = 4;  // pieces per wave per half-stage
  static_assert(C::XSZ == SL && C::WSZ == SL && C::XQ == PPH && C::WQ == PPH && C::BC / C::RPP == NW * PPH,
                "ring slot = one operand of one K-step, 4 pieces per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  const int G = gridDim.x;
  const int g = blockIdx.x & 7, i8 = blockIdx.x >> 3;
  const int q8 = G >> 3, r8 = G & 7;
  const int b = (g < r8 ? g * (q8 + 1) : r8 * (q8 + 1) + (g - r8) * q8) + i8;
  const int npix = p.n * p.oh * p.ow;
  const int nk = (p.c + 63) / 64;
  const int my_tiles = b < n_tiles ? (n_tiles - 1 - b) / G + 1 : 0;
  const int njobs = my_tiles * nk;
  if (njobs == 0) return;

  const int lrow = lane / C::NCH, lch = lane % C::NCH;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)wbytes, 0x00020000);
  const unsigned long long ybytes =
      ((unsigned long long)p.n * p.yh * p.yw - 1) * (unsigned long long)p.y_ld * 2ull + (unsigned long long)p.cout * 2ull;
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.y, 0, (int)ybytes, 0x00020000);
  // (no bias: a zero-length range, every load returns zeros)
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, 0, p.bias ? p.cout * 4 : 0, 0x00020000);

  // per-lane DMA geometry, once: piece q row (the same for both operands) and its byte offset
  // within a row block (channel chunk swizzled); the per-issue part is wave-uniform
  int prow[PPH];
  unsigned xoff[PPH], woff[PPH], chk[PPH];
#pragma unroll
  for (int q = 0; q < PPH; ++q) {
    const int row = (wave + NW * q) * C::RPP + lrow;
    const int cs = lch ^ C::swz(row);
    prow[q] = row;
    chk[q] = (unsigned)cs * 8u;
    xoff[q] = (unsigned)row * (unsigned)p.x_ld * 2u + (unsigned)cs * 16u;
    woff[q] = (unsigned)row * (unsigned)p.kpad * 2u + (unsigned)cs * 16u;
  }
  // a cursor over this workgroup's jobs (tile i, K-step k), advanced one job at a time
  struct Cur {
    int i, k, c0, p0;
  };
  auto cur_at = [&](int jj) {  // (divisions: a few times per workgroup)
    Cur c;
    c.i = jj / nk;
    c.k = jj - c.i * nk;
    const int T = b + c.i * G;
    c.c0 = (T % n_ct) * C::BC;
    c.p0 = (T / n_ct) * C::BP;
    return c;
  };
  auto cur_next = [&](Cur c) {
    if (++c.k == nk) {
      c.k = 0;
      ++c.i;
      const int T = b + c.i * G;
      c.c0 = (T % n_ct) * C::BC;
      c.p0 = (T / n_ct) * C::BP;
    }
    return c;
  };
  // operand wop of job (cursor c, live) into slot sl; a dead job (past the last) issues zero
  // pieces, so every wave's count per half-stage stays 4
  auto issue = [&](const Cur& c, bool live, int wop, int sl) {
    char* dst = smem + sl * SL + wave * 1024;
    const int cvalid = live ? p.c - 64 * c.k : 0;
    const int lim = live ? (wop ? p.cout - c.c0 : npix - c.p0) : 0;
    const unsigned base = wop ? (unsigned)c.c0 * (unsigned)p.kpad * 2u + 128u * (unsigned)c.k
                              : (unsigned)c.p0 * (unsigned)p.x_ld * 2u + 128u * (unsigned)c.k;
#pragma unroll
    for (int q = 0; q < PPH; ++q) {
      const bool ok = prow[q] < lim && (cvalid >= 64 || (int)chk[q] < cvalid);
      const unsigned o = ok ? base + (wop ? woff[q] : xoff[q]) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : rx, (lds_ptr_1x1)(dst + q * NW * 1024), 16, o, 0, 0, 0);
    }
  };

  const int wp = wave % NWP, wc = wave / NWP;
  int xf[C::NSL], wf[C::NSL];
#pragma unroll
  for (int sl = 0; sl < C::NSL; ++sl) {
    const int pr = wp * 32 * MI + r32;
    xf[sl] = pr * C::RB + (((2 * sl + hh) ^ C::swz(pr)) << 4);
    wf[sl] = (wc * 32 * TMC + r32) * C::RB + (((2 * sl + hh) ^ C::swz(r32)) << 4);
  }
  // the bias of a lane in accumulator layout: rows 8 u + 4 hh + 0..3 of 32-channel block j
  const int bco = wc * 32 * TMC + 4 * hh;

  f32x16 acc[MI][TMC];
  // prologue: half-stages 0 (x of job 0), 1 (w of job 0), 2 (x of job 1)
  Cur cj = cur_at(0);                // the job being computed
  Cur cw = cur_next(cj);             // the job whose weights issue next (jj + 1)
  Cur cx = cur_next(cw);             // the job whose x rows issue next (jj + 2)
  issue(cj, true, 0, 0);
  issue(cj, true, 1, 1);
  issue(cw, 1 < njobs, 0, 2);
  int s0 = 0;  // slot of job jj's x rows (2 jj mod 5); its weights are in slot s0 + 1 mod 5
  int jj = 0;
  // one job: the counted wait + barrier, the refill of job jj - 1's slots (the weights of job
  // jj + 1 = half-stage 2 jj + 3, the x rows of job jj + 2 = 2 jj + 4), the bias at a tile's
  // first job (loaded before the refill, so waiting for it drains nothing), the MFMAs
  auto job = [&](bool first, bool after_epi) {
    // half-stages <= 2 jj + 1 have landed (this wave's pieces by the count, the others' by the
    // barrier); only 2 jj + 2 -- plus the previous tile's epilogue stores -- may be in flight;
    // every wave's reads of job jj - 1's slots are done (lgkmcnt 0)
    if (after_epi)
      DVIE_VMCNT1(PPH + 2 * MI * TMC);
    else
      DVIE_VMCNT1(PPH);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    f32x4 bi[TMC][4];
    if (first) {
#pragma unroll
      for (int j = 0; j < TMC; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int co = cj.c0 + bco + 32 * j + 8 * u;
          // (a buffer load with an out-of-range offset past cout: zeros, no branch)
          bi[j][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, co < p.cout ? (unsigned)co * 4u : OOB, 0, 0));
        }
    }
    if (!(dbg & 4)) {
      const int sw = s0 + 3 >= NSLOT ? s0 + 3 - NSLOT : s0 + 3, sx = s0 + 4 >= NSLOT ? s0 + 4 - NSLOT : s0 + 4;
      issue(cw, jj + 1 < njobs, 1, sw);
      issue(cx, jj + 2 < njobs, 0, sx);
    }
    if (first) {
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < TMC; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[ii][j][e] = bi[j][e >> 2][e & 3];
    }
    const char* X = smem + s0 * SL;
    const char* W = smem + (s0 + 1 >= NSLOT ? s0 + 1 - NSLOT : s0 + 1) * SL;
#pragma unroll
    for (int sl = 0; sl < C::NSL; ++sl) {
      if (dbg & 2) break;
      i32x4 bq[MI], a[TMC];
#pragma unroll
      for (int ii = 0; ii < MI; ++ii) bq[ii] = *(const i32x4*)(X + xf[sl] + ii * 32 * C::RB);
#pragma unroll
      for (int j = 0; j < TMC; ++j) a[j] = *(const i32x4*)(W + wf[sl] + j * 32 * C::RB);
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < TMC; ++j)
          acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[j]),
                                                               __builtin_bit_cast(bf16x8, bq[ii]), acc[ii][j], 0, 0, 0);
    }
    s0 = s0 + 2 >= NSLOT ? s0 + 2 - NSLOT : s0 + 2;
    cj = cw;
    cw = cx;
    cx = cur_next(cx);
    ++jj;
  };
  for (int it = 0; it < my_tiles; ++it) {
    const int c0 = cj.c0, p0 = cj.p0;
    // the tile's first K-step peeled off its loop: the accumulators start from the bias there
    // and stay in place through the loop (no branch merges them)
    job(true, it > 0);
    for (int k = 1; k < nk; ++k) job(false, false);

    // ---- epilogue of tile T: activation, bf16 stores (2 MI TMC per lane), output placement
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      const int pix0 = p0 + wp * 32 * MI + 32 * ii + r32;
      const bool pix_ok = pix0 < npix;
      const int pix = pix_ok ? pix0 : npix - 1;
      long long yp = pix;
      if (p.osy != 1 || p.osx != 1 || p.ory != 0 || p.orx != 0 || p.yh != p.oh || p.yw != p.ow) {
        const int hw = p.oh * p.ow;
        const int n = pix / hw, r = pix - n * hw;
        const int oy = r / p.ow, ox = r - oy * p.ow;
        yp = ((long long)n * p.yh + oy * p.osy + p.ory) * p.yw + ox * p.osx + p.orx;
      }
#pragma unroll
      for (int j = 0; j < TMC; ++j)
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          float w[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[ii][j][8 * P + e]),
                                                             __float_as_uint(acc[ii][j][8 * P + 4 + e]), false, false);
            w[e] = __uint_as_float(sw[0]);
            w[4 + e] = __uint_as_float(sw[1]);
          }
          if (ACT == DVIE_ACT_LRELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = fmaxf(w[e], w[e] * p.alpha);  // (0 <= alpha <= 1: launch)
          }
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (int)pk_bf16(w[2 * e], w[2 * e + 1]);
          const int co = c0 + wc * 32 * TMC + 32 * j + 16 * P + 8 * hh;
          // (a buffer store that every wave issues, out-of-range lanes aimed past the buffer's
          // range and dropped: the per-wave store count the next wait counts on is uniform)
          const unsigned yo = (pix_ok && co < p.cout && !(dbg & 1)) ? (unsigned)((yp * p.y_ld + co) * 2) : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), ry, yo, 0, 0);
        }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// operand sets instantiated per tile shape: single K-step, at most 4 accumulators per wave
// (a single prefetched operand on the 8-accumulator 64->256 tile measured no gain)
template <int V, int NS, int MT>
struct PreOk {
  static constexpr int v = NS != 1 || MT > 4 ? 0 : V;
};

// DVIE_1X1_PERSIST=0: one tile per workgroup for multi-K-step layers (A/B runs); read per launch
static bool persist_env_on() {
  const char* e = getenv("DVIE_1X1_PERSIST");
  return !(e && *e == '0');
}

// DVIE_1X1_DBG (timing only, wrong results; -DDVIE_TIMING_DBG builds only): bit 1 skips the epilogue stores, bit 2 the
// MFMA loop (operand DMA kept); read per launch
static int dbg_env() {
#ifdef DVIE_TIMING_DBG
  const char* e = getenv("DVIE_1X1_DBG");
  return e && *e ? atoi(e) : 0;
#else
  return 0;
#endif
}

// DVIE_1X1_RING=0: the wide multi-K-step layers on the two-stage kernel (A/B runs); read per launch
static bool ring_env_on() {
  const char* e = getenv("DVIE_1X1_RING");
  return !(e && *e == '0');
}

// DVIE_1X1_CE=0: the MFMA-layout epilogue stores for the single-K-step wide tiles (A/B runs);
// read per launch
static bool ce_env_on() {
  const char* e = getenv("DVIE_1X1_CE");
  return !(e && *e == '0');
}

// DVIE_1X1_PRE=0: no epilogue-operand prefetch (A/B runs); read per launch
static bool pre_env_on() {
  const char* e = getenv("DVIE_1X1_PRE");
  return !(e && *e == '0');
}

template <int TMC, int NS, int KC = 64, int NWP = 8, int MI = 1, int NWC = 1>
static void launch_1x1(const dvie_conv_desc& p, hipStream_t s) {
  typedef G1Cfg<TMC, NS, KC, NWP, MI, NWC> C;
  constexpr int NW = C::NW;
  const int npix = p.n * p.oh * p.ow;
  const int n_ct = (p.cout + C::BC - 1) / C::BC;
  const int n_tiles = n_ct * ((npix + C::BP - 1) / C::BP);
  if (p.out_f32) {
    DVIE_LAUNCH((conv1x1_kernel<TMC, NS, KC, NWP, MI, NWC, true>), dim3(n_tiles), dim3(64 * NW), 0, s, p, n_ct, n_tiles, dbg_env());
    return;
  }
  if constexpr (NS == 2 && KC == 64 && TMC == 4 && NWP == 4 && MI == 2 && NWC == 2) {
    // the wide multi-K-step layers without epilogue operands: the five-slot operand ring
    const unsigned long long span = ((unsigned long long)p.n * p.yh * p.yw - 1) * (unsigned long long)p.y_ld * 2ull +
                                    (unsigned long long)p.cout * 2ull;
    const unsigned long long xspan = ((unsigned long long)npix - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
    if (ring_env_on() && p.c > KC && n_tiles > 256 && !p.res && !p.beta && !p.dact && span < 0xFFFFFF00ull &&
        xspan < 0xFFFFFF00ull && p.ih == p.oh && p.iw == p.ow &&
        (p.act == DVIE_ACT_NONE || (p.act == DVIE_ACT_LRELU && p.alpha >= 0.f && p.alpha <= 1.f))) {
#ifdef DVIE_TIMING_DBG
      if (p.act == DVIE_ACT_LRELU) switch (dbg_env() & 7) {
#define DVIE_RING_AB(V)                                                                                                \
  case V:                                                                                                              \
    DVIE_LAUNCH((conv1x1_ring_kernel<TMC, NWP, MI, NWC, DVIE_ACT_LRELU, V>), dim3(256), dim3(64 * NW), 0, s, p, n_ct, \
                n_tiles);                                                                                              \
    return;
          DVIE_RING_AB(1) DVIE_RING_AB(2) DVIE_RING_AB(3) DVIE_RING_AB(4) DVIE_RING_AB(5) DVIE_RING_AB(6) DVIE_RING_AB(7)
#undef DVIE_RING_AB
          default: break;
        }
#endif
      if (p.act == DVIE_ACT_LRELU)
        DVIE_LAUNCH((conv1x1_ring_kernel<TMC, NWP, MI, NWC, DVIE_ACT_LRELU>), dim3(256), dim3(64 * NW), 0, s, p, n_ct, n_tiles);
      else
        DVIE_LAUNCH((conv1x1_ring_kernel<TMC, NWP, MI, NWC, DVIE_ACT_NONE>), dim3(256), dim3(64 * NW), 0, s, p, n_ct, n_tiles);
      return;
    }
  }
  if constexpr (NS >= 2 && NS <= 5 && MI * TMC <= 4) {
    // several K-steps and more tiles than resident workgroups: persistent stage ring
    // (8x256x512 256->64: 142 -> 127 us, 8x128x256 256->128: 47 -> 41 us; the 8-accumulator
    // wide tiles of the heads measured no gain, 896->448 +3%: they keep one tile per workgroup)
    const int per_cu = 163840 / C::SMEM;
    const int G = 256 * (per_cu > 2 ? 2 : per_cu);
    if (persist_env_on() && p.c > KC && n_tiles > G) {
      DVIE_LAUNCH((conv1x1_persist_kernel<TMC, NS, KC, NWP, MI, NWC>), dim3(G), dim3(64 * NW), 0, s, p, n_ct,
                         n_tiles);
      return;
    }
  }
  // single K-step with identity placement: prefetch the epilogue operands (all of them when
  // the registers allow -- MI * TMC <= 4 -- else the activation input, or the residual)
  const bool ident = p.osy == 1 && p.osx == 1 && p.ory == 0 && p.orx == 0 && p.yh == p.oh && p.yw == p.ow;
  int pre = 0;
  if constexpr (NS == 1) {
    if (ident && p.c <= KC && pre_env_on()) {
      pre = MI * TMC > 4 ? 0 : (p.res ? 1 : 0) | (p.beta ? 2 : 0) | (p.dact ? 4 : 0);
    }
  }
  if constexpr (NS == 1 && MI == 1 && 2 * TMC == 8) {
    if (ident && ce_env_on() && p.cout % C::BC == 0) {
      switch (pre) {
#define DVIE_1X1_CE_CASE(V)                                                                                          \
  case V:                                                                                                            \
    DVIE_LAUNCH((conv1x1_kernel<TMC, NS, KC, NWP, MI, NWC, false, PreOk<V, NS, MI * TMC>::v, true>), dim3(n_tiles), \
                       dim3(64 * NW), 0, s, p, n_ct, n_tiles, 0);                                                     \
    return;
        DVIE_1X1_CE_CASE(0) DVIE_1X1_CE_CASE(1) DVIE_1X1_CE_CASE(2) DVIE_1X1_CE_CASE(3) DVIE_1X1_CE_CASE(4)
        DVIE_1X1_CE_CASE(5) DVIE_1X1_CE_CASE(6) DVIE_1X1_CE_CASE(7)
#undef DVIE_1X1_CE_CASE
      }
    }
  }
  switch (pre) {
#define DVIE_1X1_PRE_CASE(V)                                                                                      \
  case V:                                                                                                        \
    DVIE_LAUNCH((conv1x1_kernel<TMC, NS, KC, NWP, MI, NWC, false, PreOk<V, NS, MI * TMC>::v>), dim3(n_tiles), \
                       dim3(64 * NW), 0, s, p, n_ct, n_tiles, dbg_env());                                                   \
    break;
    DVIE_1X1_PRE_CASE(1) DVIE_1X1_PRE_CASE(2) DVIE_1X1_PRE_CASE(3) DVIE_1X1_PRE_CASE(4) DVIE_1X1_PRE_CASE(5)
    DVIE_1X1_PRE_CASE(6) DVIE_1X1_PRE_CASE(7)
#undef DVIE_1X1_PRE_CASE
    default:
      DVIE_LAUNCH((conv1x1_kernel<TMC, NS, KC, NWP, MI, NWC, false>), dim3(n_tiles), dim3(64 * NW), 0, s, p, n_ct, n_tiles, dbg_env());
  }
}

// Returns true when the 1x1 GEMM kernel took the launch.
bool conv1x1_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (p.dtype != DVIE_BF16 || p.th != 1 || p.tw != 1) return false;
  if (p.sy != 1 || p.sx != 1 || p.dy0 != 0 || p.dx0 != 0 || p.ih != p.oh || p.iw != p.ow) return false;
  if (p.osy < 1 || p.osx < 1 || p.ory < 0 || p.orx < 0) return false;
  if (p.c % 64 != 0 && p.c > 64) return false;
  if ((long long)p.n * p.oh * p.ow >= (1LL << 31)) return false;
  const char* e = getenv("DVIE_CONV_CFG");
  int cfg = e && *e ? atoi(e) : -3;
  if (cfg >= 0 && cfg < 100) return false;  // tuning override forces the halo / per-tap kernels
  const int cout = p.cout;
  const bool one = p.c <= 64;  // a single K-step: one stage, several workgroups per CU

  // wide layers: 2-D wave grid (116; 448->448 heads 724 -> 662 us, 64->256 166 -> 155 us
  // at 8x256x512, tools/conv_tune.py)
  // (DVIE_CONV1X1_WIDE overrides the wide-layer choice alone, for A/B runs of the whole step)
  static const int wide = getenv("DVIE_CONV1X1_WIDE") && *getenv("DVIE_CONV1X1_WIDE") ? atoi(getenv("DVIE_CONV1X1_WIDE")) : 116;
  // single K-step, 65-128 output channels: two 64-channel column tiles with every epilogue
  // operand prefetched beat one 128-channel tile (8x128x256 64->128: 33 vs 35 us residual,
  // 48 vs 56 us accumulate + activation input, tools/conv_epi_micro.py)
  // single K-step wide layers (layer1's 64->256 forward, the 256-channel data gradients of its
  // 256->64 convs): 128-channel wave tiles of 4 accumulators with every epilogue operand
  // prefetched (101) beat the 2-D wave grid's 8 (116): 213.5 -> 214.7 frames/s, 5 of 6 same-box
  // pairs (profiles/r03wide1/); DVIE_CONV1X1_WIDE1 overrides it (A/B runs)
  static const int wide1 = getenv("DVIE_CONV1X1_WIDE1") && *getenv("DVIE_CONV1X1_WIDE1") ? atoi(getenv("DVIE_CONV1X1_WIDE1")) : 101;
  if (cfg < 0) cfg = cout <= 64 ? 100 : cout <= 128 ? (one ? 100 : 101) : one ? wide1 : wide;
  switch (cfg) {
    case 100: one ? launch_1x1<2, 1>(p, s) : launch_1x1<2, 3>(p, s); break;
    case 101: one ? launch_1x1<4, 1>(p, s) : launch_1x1<4, 3>(p, s); break;
    case 102: one ? launch_1x1<7, 1>(p, s) : launch_1x1<7, 2>(p, s); break;
    case 103: one ? launch_1x1<8, 1>(p, s) : launch_1x1<8, 2>(p, s); break;
    case 104: one ? launch_1x1<4, 1>(p, s) : launch_1x1<4, 2>(p, s); break;
    // 32-channel K-steps: deeper pipelines in the same LDS (measured: no gain, the kernel is
    // not load-latency bound)
    case 105: one ? launch_1x1<7, 1>(p, s) : launch_1x1<7, 4, 32>(p, s); break;
    case 106: one ? launch_1x1<7, 1>(p, s) : launch_1x1<7, 5, 32>(p, s); break;
    // 4-wave workgroups (128-pixel tiles, two workgroups per CU)
    case 110: one ? launch_1x1<7, 1, 64, 4>(p, s) : launch_1x1<7, 2, 32, 4>(p, s); break;
    // 2-D wave grids: 64-pixel x 128-channel wave tiles (6 fragments per 8 MFMAs)
    case 116: one ? launch_1x1<4, 1, 64, 4, 2, 2>(p, s) : launch_1x1<4, 2, 64, 4, 2, 2>(p, s); break;
    case 118: one ? launch_1x1<2, 1, 64, 4, 2, 2>(p, s) : launch_1x1<2, 3, 64, 4, 2, 2>(p, s); break;
    case 119: one ? launch_1x1<4, 1, 64, 4, 2, 2>(p, s) : launch_1x1<4, 4, 32, 4, 2, 2>(p, s); break;
    case 120: one ? launch_1x1<4, 1, 64, 4, 2, 2>(p, s) : launch_1x1<4, 5, 32, 4, 2, 2>(p, s); break;
    default: return false;
  }
  return true;
}

}  // namespace dvie
