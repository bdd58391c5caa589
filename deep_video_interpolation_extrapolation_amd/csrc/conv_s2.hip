// Stride-2 3x3 forward convolution (zero padding 1) for gfx950, bf16: HRNet's downsampling
// convs -- transition1.1 / transition2.2 and the strided fuse-layer chains (reference
// nets/HRNet.py:166-194 fuse_layers, l.444-477 transition layers).
//
// Phase-split halo.  A workgroup owns PR = 4 output rows x 64 output pixels x BC output
// channels.  Its input region, (2 PR + 1) rows x 129 columns, is staged once per 16-channel
// chunk by LDS-DMA, each input row split into its even and its odd columns (two "phase rows"
// of 65 pixels): output pixel j's tap (ti, tj) reads input column 2j + tj - 1, i.e. pixel
// j + (tj >> 1) of phase row tj & 1, so the B fragment of a tap for 32 consecutive output
// pixels is 32 consecutive pixels of one phase row -- a stride-1 read, as in the stride-1
// halo kernels, and the input is fetched once per chunk instead of once per tap (the per-tap
// implicit GEMM of conv_fwd.hip gathered it nine times from L2).  Pixel pitch 32 B (16
// channels), the two 16-B halves of pixel p swapped when bit 3 of p is set: any 16
// consecutive pixels' b128 reads hit 16 distinct bank quads, and no DMA lane is spent on pad.
//   Weights stream one tap COLUMN (3 taps, BC rows x 32 B each, 16-B chunks XOR-swizzled by
// (row >> 3) & 1) per step through a ring of three column buffers, issued two steps ahead;
// the next chunk's halo is issued in two shares under the current chunk's first two columns.
// One vmcnt wait + barrier per column; the wait leaves the two younger weight columns and the
// halo shares that are not yet needed in flight.
//   8 MFMA waves = 2 (output-channel halves of 32 TM) x 4 (output rows); a wave owns 32 TM
// channels x 1 row x 64 pixels (2 TM accumulators of 32 x 32).  Two more waves
// issue all the LDS-DMA (TM = 2; the MFMA waves then never stall behind the address unit).  LDS:
// 2 x 40 KB halo + 3 column buffers (8 / 16 / 24 KB for TM = 1 / 2 / 4): one workgroup per
// CU, persistent over an XCD-contiguous tile range.  Epilogue from registers: bias, residual
// (EPI bit 1), activation.
//   What bounds it (8x256x512 256->128, tools/s2_ab.sh + tools/pmc_s2.sh, r05): 275 us with
// the MFMA waves issuing the DMA, TA busy ~70% of the kernel; with every DMA removed
// (timing-only build) 121 us; weights as one contiguous block per column -8%, dedicated DMA
// waves -5%, both -15%.  The 32-B-per-pixel (16-channel) fragment loads cost the address
// unit ~4x the cycles of whole 128-B lines; wider chunks need a halo that no longer fits
// double-buffered beside the weight ring.
#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_s2;

// vmcnt(N) and lgkmcnt(0)
#define DVIE_S2_VMCNT_LGKM0(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4))

__device__ __forceinline__ uint32_t s2_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

template <int TM, int DW>
struct S2 {
  static constexpr int NWM = 8;                    // MFMA waves
  static constexpr int NI = DW ? DW : NWM;         // DMA-issuing waves (DW > 0: dedicated ones)
  static constexpr int NTH = 64 * (NWM + DW);
  static constexpr int BC = 64 * TM, PR = 4, KC = 16;
  static constexpr int HR = 2 * PR + 1, HP = 65;  // halo rows; pixels per phase row
  static constexpr int RSLOTS = 2 * HP * 2;        // 16-B slots per input row (two phase rows)
  static constexpr int HSLOTS = HR * RSLOTS;
  static constexpr int NHI = ((HSLOTS + 63) / 64 + NI - 1) / NI * NI;
  static constexpr int NHQ = NHI / NI;             // halo pieces per issuing wave per chunk
  static constexpr int HSZ = NHI * 1024;
  static constexpr int TSZ = BC * 32;              // one tap of one chunk: BC rows x 32 B
  static constexpr int WP = 3 * TSZ / 1024;        // weight pieces per column
  static constexpr int WPC = (WP + NI - 1) / NI;   // weight pieces per issuing wave per column
  static constexpr int WSZ = WPC * NI * 1024;      // one column buffer
  static constexpr int SMEM = 2 * HSZ + 3 * WSZ;
  static constexpr int H0 = NHQ * 3 / 5;           // halo pieces per issuing wave in column 0 (rest: column 1)
};
static_assert(S2<4, 0>::SMEM <= 163840 && S2<2, 2>::SMEM <= 163840, "conv_s2 LDS budget");
static_assert(S2<2, 0>::NHQ == 5 && S2<2, 0>::H0 == 3, "halo shares");
static_assert(S2<2, 2>::WPC + S2<2, 2>::NHQ < 64 && S2<4, 0>::WPC + S2<4, 0>::NHQ < 64, "vmcnt range");

struct S2Job {
  int valid, t, k, c0, n, y0, x0;
};

// halo pieces [qa, qb) of job J (piece i of this wave at dst + i * NI KB; a job past the end
// issues its pieces with an empty range: they land as zeros nobody reads, and the vmcnt
// bookkeeping stays compile-time)
template <int NI>
__device__ __forceinline__ void s2_halo(const dvie_conv_desc& p, const S2Job& J, char* dst, const int* hgeo, int qa,
                                        int qb, unsigned long long xbytes, unsigned xrow) {
  const unsigned OOB = 0xFFFFFFF0u;
  const int nrec = J.valid ? (int)(xbytes - (unsigned long long)J.k * 32) : 0;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.x + (size_t)J.k * 32), 0, nrec, 0x00020000);
  const int ybase = 2 * J.y0 - 1, xbase = 2 * J.x0 - 1;
#pragma unroll
  for (int q = qa; q < qb; ++q) {
    const int gq = hgeo[q];
    const int iy = ybase + (gq >> 16), ix = xbase + ((gq >> 4) & 0xFFF);
    const bool ok = gq >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
    const unsigned o0 = (unsigned)((J.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(gq & 15) * 16u;
    const unsigned o = ok ? o0 : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_s2)(dst + q * NI * 1024), 16, o, 0, 0, 0);
  }
}

// DW: dedicated DMA waves (0: the MFMA waves issue the LDS-DMA themselves)
template <int TM, int EPI, int DW>
__global__ __launch_bounds__(64 * (8 + DW)) void conv_s2_kernel(const dvie_conv_desc p, int n_ct, int n_tiles,
                                                                int tiles_x, int tiles_y) {
  typedef S2<TM, DW> C;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool is_mma = DW == 0 || wave < C::NWM, is_dma = DW == 0 || wave >= C::NWM;
  const int dwave = DW ? (wave >= C::NWM ? wave - C::NWM : 0) : wave;  // issuing-wave index
  const int wc = (wave >> 2) & 1, wr = wave & 3;
  const int r32 = lane & 31, hh = lane >> 5;
  const int nchunks = p.c >> 4;
  const unsigned OOB = 0xFFFFFFF0u;

  // persistent: XCD g (= blockIdx % 8) takes a contiguous tile range, its blocks stride it
  const int G = gridDim.x, g = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nbg = G / 8 + (g < G % 8 ? 1 : 0);
  const int q8 = n_tiles / 8, r8 = n_tiles % 8;
  const int ts = g < r8 ? g * (q8 + 1) : r8 * (q8 + 1) + (g - r8) * q8;
  const int tile0 = ts + jb, tile_end = ts + q8 + (g < r8 ? 1 : 0);
  if (tile0 >= tile_end) return;

  auto tile_job = [&](int t) {
    S2Job J;
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
  auto next_job = [&](const S2Job& J) {
    if (J.k + 1 < nchunks) {
      S2Job N = J;
      N.k = J.k + 1;
      return N;
    }
    return tile_job(J.t + nbg);
  };

  // halo DMA geometry: slot -> (input row hr, input column hc = 2 px + phase, 16-B half cs;
  // the halves of pixel px swapped when bit 3 of px is set)
  int hgeo[C::NHQ];
#pragma unroll
  for (int q = 0; q < C::NHQ; ++q) {
    const int slot = (dwave + C::NI * q) * 64 + lane;
    const int hr = slot / C::RSLOTS, rem = slot - (slot / C::RSLOTS) * C::RSLOTS;
    const int ph = rem / (2 * C::HP), rem2 = rem - ph * (2 * C::HP);
    const int px = rem2 >> 1, cs = (rem2 & 1) ^ ((px >> 3) & 1);
    hgeo[q] = slot < C::HSLOTS ? (hr << 16) | ((2 * px + ph) << 4) | cs : -1;
  }
  // weight DMA geometry: slot -> (tap row ti of the column, weight row, source chunk); the
  // source offset without the per-issue terms (channel block, column, chunk), or OOB
  unsigned woff[C::WPC];
#pragma unroll
  for (int q = 0; q < C::WPC; ++q) {
    const int slot = (dwave + C::NI * q) * 64 + lane;
    const int ti = slot / (2 * C::BC), rem = slot - ti * (2 * C::BC);
    const int row = rem >> 1, ch = (rem & 1) ^ ((row >> 3) & 1);
    const unsigned wo = (unsigned)row * (unsigned)p.kpad * 2u + (unsigned)(ti * 3 * p.c + ch * 8) * 2u;
    woff[q] = slot < 3 * 2 * C::BC ? wo : OOB;
  }
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;

  char* const Hs = smem;
  char* const As = smem + 2 * C::HSZ;  // column v of a job in buffer v

  // halo pieces [qa, qb) of job J into halo buffer hb (s2_halo above)
  auto halo_issue = [&](const S2Job& J, int hb, int qa, int qb) {
    s2_halo<C::NI>(p, J, Hs + hb * C::HSZ + dwave * 1024, hgeo, qa, qb, xbytes, xrow);
  };
  // tap column v of job J into column buffer ab (all non-lane terms in the resource base)
  auto a_issue = [&](const S2Job& J, int v, int ab) {
    const unsigned o = (unsigned)(J.c0 * p.kpad + v * p.c + 16 * J.k) * 2u;
    const int nrec = J.valid ? (int)(wbytes - o) : 0;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.w + o), 0, nrec, 0x00020000);
    char* dst = As + ab * C::WSZ + dwave * 1024;
#pragma unroll
    for (int q = 0; q < C::WPC; ++q) {
      // (the offset as a statement of its own: an array element passed straight to the
      // builtin makes hipcc's host pass drop the kernel's launch stub)
      const unsigned wo = woff[q];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_s2)(dst + q * C::NI * 1024), 16, wo, 0, 0, 0);
    }
  };

  // fragment addresses: A row wc*32*TM + 32 i + r32 (chunk hh, swizzled); B pixel 32 b + r32 + s
  // (s = v >> 1) of phase row (2 wr + ti, v & 1), channel half hh (swapped by bit 3 of the pixel)
  int a_off[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wc * 32 * TM + 32 * i + r32;
    a_off[i] = row * 32 + ((hh ^ ((row >> 3) & 1)) << 4);
  }
  int b_off[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int px = r32 + s;
    b_off[s] = (2 * wr * 2 * C::HP) * 32 + px * 32 + ((hh ^ ((px >> 3) & 1)) << 4);
  }

  f32x16 acc[TM][2];

  {
    const S2Job J0 = tile_job(tile0);
    if (is_dma) {
      halo_issue(J0, 0, 0, C::NHQ);
      a_issue(J0, 0, 0);
      a_issue(J0, 1, 1);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  int hb = 0;
  S2Job J = tile_job(tile0);
  S2Job J1 = next_job(J);
  while (J.valid) {
    if (J.k == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][b][e] = 0.f;
    }
    const char* H = Hs + hb * C::HSZ;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const char* A = As + v * C::WSZ;
      // DMA, two steps ahead: the weights of the column after next (this job's column 2, then
      // the next job's columns 0 and 1) into the buffer read in the previous step, then this
      // column's share of the next job's halo
      if (is_dma) {
        if (v == 0)
          a_issue(J, 2, 2);
        else
          a_issue(J1, v - 1, v - 1);
        if (v == 0) halo_issue(J1, hb ^ 1, 0, C::H0);
        if (v == 1) halo_issue(J1, hb ^ 1, C::H0, C::NHQ);
      }
      if (is_mma) {
        const char* Hv = H + b_off[v >> 1] + (v & 1) * C::HP * 32;
        i32x4 af[3][TM], bf[3][2];
#pragma unroll
        for (int ti = 0; ti < 3; ++ti) {
#pragma unroll
          for (int i = 0; i < TM; ++i) af[ti][i] = *(const i32x4*)(A + ti * C::TSZ + a_off[i]);
#pragma unroll
          for (int b = 0; b < 2; ++b) bf[ti][b] = *(const i32x4*)(Hv + (ti * 2 * C::HP + 32 * b) * 32);
        }
#pragma unroll
        for (int ti = 0; ti < 3; ++ti)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[i][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[ti][i]),
                                                                  __builtin_bit_cast(bf16x8, bf[ti][b]), acc[i][b], 0,
                                                                  0, 0);
      }
      // end of the column: the next column's weights (and after column 2 the next job's whole
      // halo) have landed -- what was issued after them may stay in flight -- and every wave's
      // reads of this column's buffers are done (lgkmcnt 0), so they may be refilled after the
      // barrier
      if (is_dma) {
        if (v == 0)
          DVIE_S2_VMCNT_LGKM0(C::WPC + C::H0);
        else if (v == 1)
          DVIE_S2_VMCNT_LGKM0(C::WPC + C::NHQ);
        else
          DVIE_S2_VMCNT_LGKM0(C::WPC);
      } else {
        __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (3 << 14));  // lgkmcnt(0)
      }
      __builtin_amdgcn_s_barrier();
    }
    hb ^= 1;

    if (is_mma && J.k + 1 == nchunks) {
      // ---- epilogue from the accumulators: permlane32_swap pairs the half-waves so that each
      // lane owns 8 consecutive channels of one pixel ----
      const int oy = J.y0 + wr;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          float v8[2][8];
#pragma unroll
          for (int P = 0; P < 2; ++P)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][b][8 * P + e]),
                                                               __float_as_uint(acc[i][b][8 * P + 4 + e]), false, false);
              v8[P][e] = __uint_as_float(sw[0]);
              v8[P][4 + e] = __uint_as_float(sw[1]);
            }
          const int ox = J.x0 + 32 * b + r32;
          if (oy >= p.oh || ox >= p.ow) continue;
          const long long pix = ((long long)J.n * p.yh + oy) * p.yw + ox;
#pragma unroll
          for (int P = 0; P < 2; ++P) {
            const int co = J.c0 + wc * 32 * TM + 32 * i + 16 * P + 8 * hh;
            if (co >= p.cout) continue;
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
              const i32x4 tr = *(const i32x4*)((const bf16_t*)p.res + pix * p.res_ld + co);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[2 * e] += __uint_as_float(((uint32_t)tr[e]) << 16);
                w[2 * e + 1] += __uint_as_float(((uint32_t)tr[e]) & 0xffff0000u);
              }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = act_bf(w[e], p.act, p.alpha);
            i32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (int)s2_pack(w[2 * e], w[2 * e + 1]);
            *(i32x4*)((bf16_t*)p.y + pix * p.y_ld + co) = o;
          }
        }
    }
    J = J1;
    J1 = next_job(J1);
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// TM = 2: two dedicated DMA waves beside the eight MFMA waves (8x256x512 256->128:
// 276 -> 262 us, tools/s2_ab.sh; 8x128x256 64->64, TM = 1: 21.9 us without, 23.2 with them);
// TM = 4 has no registers for a third wave per SIMD.  (Hoisting every fragment read of a
// column ahead of its MFMAs with a scheduling barrier: 262 -> 287 us, not kept.)
template <int TM>
static void launch_s2(const dvie_conv_desc& p, hipStream_t s) {
  constexpr int DW = TM == 2 ? 2 : 0;
  typedef S2<TM, DW> C;
  const int n_ct = (p.cout + C::BC - 1) / C::BC;
  const int tiles_x = (p.ow + 63) / 64, tiles_y = (p.oh + C::PR - 1) / C::PR;
  const int n_tiles = n_ct * tiles_x * tiles_y * p.n;
  const int grid = n_tiles > 256 ? 256 : n_tiles;
  if (p.res)
    DVIE_LAUNCH((conv_s2_kernel<TM, 1, DW>), dim3(grid), dim3(C::NTH), 0, s, p, n_ct, n_tiles, tiles_x, tiles_y);
  else
    DVIE_LAUNCH((conv_s2_kernel<TM, 0, DW>), dim3(grid), dim3(C::NTH), 0, s, p, n_ct, n_tiles, tiles_x, tiles_y);
}

// DVIE_CONV_S2=0: stride-2 convs on the per-tap implicit GEMM (A/B runs); read per launch
static bool s2_on() {
  const char* e = getenv("DVIE_CONV_S2");
  return !(e && *e == '0');
}

// stride-2 3x3 zero-padded forward conv, bf16 output, identity output placement; true when
// the phase-split halo kernel took the launch
bool conv_s2_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (!s2_on() || p.dtype != DVIE_BF16 || p.out_f32 || p.beta || p.dact) return false;
  if (p.sy != 2 || p.sx != 2 || p.th != 3 || p.tw != 3 || p.dy0 != -1 || p.dx0 != -1 || p.ddy != 1 || p.ddx != 1)
    return false;
  if (p.osy != 1 || p.osx != 1 || p.ory != 0 || p.orx != 0 || p.yh != p.oh || p.yw != p.ow) return false;
  if (p.c % 16 != 0 || p.cout % 8 != 0 || p.kpad < 9 * p.c) return false;
  if ((p.res && (p.res_ld % 8 != 0 || ((uintptr_t)p.res & 15) != 0)) || p.y_ld % 8 != 0 || p.x_ld % 8 != 0) return false;
  const unsigned long long pix = (unsigned long long)p.n * p.ih * p.iw;
  if (((pix - 1) * (unsigned long long)p.x_ld + (unsigned long long)p.c) * 2ull >= 0xFFFFFF00ull) return false;
  if ((unsigned long long)p.cout * p.kpad * 2ull >= 0xFFFFFF00ull) return false;
  // expected output grid of a pad-1 stride-2 3x3 conv
  if (p.oh != (p.ih - 1) / 2 + 1 || p.ow != (p.iw - 1) / 2 + 1) return false;
  const long long nt = (long long)p.n * ((p.oh + 3) / 4) * ((p.ow + 63) / 64) * ((p.cout + 63) / 64);
  if (nt >= (1LL << 30)) return false;
  if (p.cout <= 64)
    launch_s2<1>(p, s);
  else if (p.cout <= 128)
    launch_s2<2>(p, s);
  else
    launch_s2<4>(p, s);
  return true;
}

}  // namespace dvie
