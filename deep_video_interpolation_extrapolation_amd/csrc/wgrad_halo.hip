// Halo-tile weight gradient for gfx950, bf16: stride-1 convolutions with a 1x1 or 3x3 tap
// grid (the weight gradient of every 3x3/1x1 stride-1 conv of HRNet/VGG).
//
//   part[slab][co][t*c + ci] = sum_{pix} g[pix][co] * x[pix + shift(t)][ci]
//
// A workgroup owns one (64 output-channel, 64 input-channel) block and a contiguous range
// of output tiles (PR rows x 64 pixels).  Per tile it stages, once, the output-gradient tile
// G [PR*64 px][64 co] and the input halo X [(PR+TH-1) x (64+TW-1) px][64 ci]; every tap reads
// its operands from those images (the per-tap kernel in conv.hip re-gathers x once per tap).
// Both images are 128-byte rows with chunk c stored at c ^ (4 * ((row >> 1) & 1)), which makes
// the ds_read_b64_tr_b16 transposed reads (4 consecutive rows x 64 B per 32-lane half)
// conflict-free at any row shift.  The next tile's images stream in (LDS-DMA, double
// buffered) while the current tile's MFMAs run; one barrier per tile.
//
// MFMA v_mfma_f32_32x32x16_bf16 with K = pixels: A = G^T (co x px), B = X (px x ci), both
// from transposed reads.  3x3: waves own (32 co x 32 ci) and all 9 taps (9 accumulators).
// 1x1: waves own the full 64 x 64 block for a quarter of the pixels and write separate
// partial slabs.  The slabs are summed by dvie_wgrad_reduce.
//
// Reference op replaced: nn.Conv2d backward-weight (nets/HRNet.py, nets/vgg.py).
#include <stdlib.h>

#include <type_traits>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_wg;

__device__ __forceinline__ bf16x8 tr_pair(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// t + the sum of a fragment's 8 bf16 values, in fp32: four v_dot2c_f32_bf16 against (1, 1)
// (bias column sums)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float sum8_bf16(const bf16x8 v, float t) {
  const i32x4 u = __builtin_bit_cast(i32x4, v);
  const bf16x2_t one = __builtin_bit_cast(bf16x2_t, 0x3F803F80);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int w = u[e];  // (a bit_cast of the vector element itself reads element 0 on this compiler)
    t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, w), one, t, false);
  }
  return t;
}

template <int TH, int TW, int PR, int TMO, int TMI>
struct WgCfg {
  static constexpr int NT = TH * TW;
  static constexpr int BCO = 64 * TMO, BCI = 64 * TMI;  // output / input channels per block
  static constexpr int HR = PR + TH - 1;                // halo rows of one tile
  static constexpr int XW = TW == 1 ? 64 : 72;          // LDS row pitch of a halo row, in pixels
  static constexpr int R = HR + PR;                     // ring: current tile + next tile's new rows
  static constexpr int GROWS = PR * 64;
  static constexpr int GPI = GROWS / 8;                 // DMA pieces (8 pixels x 128 B) per sub-image
  static constexpr int XPR = XW / 8;                    // DMA pieces per halo row
  static constexpr int GSUB = GPI * 1024;               // one 64-channel G sub-image
  static constexpr int XSUB = R * XW * 128;             // one 64-channel X ring
  static constexpr int GSZ = TMO * GSUB, XSZ = TMI * XSUB;
  static constexpr int SMEM = 2 * GSZ + XSZ;
  static constexpr int NACC = NT * TMO * TMI;
};

// Tiles walk down a column (ty fastest) so that consecutive tiles of a workgroup share
// TH-1 halo rows: the input halo lives in a ring of R = HR + PR rows, and each new tile loads
// only its PR new rows (while the current tile computes) plus its output-gradient tile.
__device__ __forceinline__ int xcd_chunk(int b, int nb) {
  // blocks b and b+8 share an XCD under round-robin dispatch: give XCD g a contiguous range
  const int g = b & 7, i = b >> 3;
  const int q = nb >> 3, r = nb & 7;
  return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}

// 8 waves: (co half, ci half, row half); the two row halves accumulate separately and are
// summed through LDS into one partial slab per split.  NW = 4 (output channels <= 32, the
// 448 -> 3 / 448 -> 20 heads): no co half -- the second half's waves would only multiply the
// zero padding of channels 32..63, and without them each wave has its SIMD's MFMA pipe alone.
//
// PIPE: the next k-step's fragments (its G fragment and all NT * TMI shifted X fragments) are
// read from LDS while the current k-step's MFMAs run (two fragment sets in registers), instead
// of each MFMA waiting on the transposed reads issued just before it.
// AB: timing-only ablations, compiled into -DDVIE_TIMING_DBG builds only (DVIE_WG_DBG): 8 = no
// DMA after the first tile (stale operands), 16 = no MFMAs, 32 = no slab stores, 64 = no LDS
// fragment reads after a tile's first two k-steps, 128 = no end-of-tile wait and barrier
// DOB (PIPE form): the bias column sums are compiled in (a launch with p.bws); without them
// the k-steps carry no v_dot2c (most HRNet convs have no bias: 4 of them per k-step per wave
// sat beside the MFMAs for nothing)
template <int TH, int TW, int PR, int TMO, int TMI, int NW = 8, bool PIPE = false, int AB = 0, bool DOB = true>
__global__ __launch_bounds__(64 * NW) void wgrad_halo_kernel(const dvie_wgrad_desc p, int n_co, int n_ci, int splits,
                                                             int tiles_x, int tiles_y, int n_tiles, int flags) {
  typedef WgCfg<TH, TW, PR, TMO, TMI> C;
  static_assert(PR % 2 == 0, "row halves");
  static_assert(NW == 8 || (NW == 4 && TMO == 1), "4-wave form: one 32-channel co block");
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int merge = flags & 1;
  constexpr int dbg = AB;  // (timing-only ablation bits, above)
  // flags bit 1: static priority for the second-dispatched half of the waves (the arbitration
  // loser on every MFMA/VALU segment, MI355X_MICROARCH "Two waves per SIMD" item 4)
  if ((flags & 2) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const unsigned OOB = 0xFFFFFFF0u;

  // all (co, ci) pairs of one split run on one XCD, so they share the split's g / x tiles in L2
  const int npair = n_co * n_ci;
  const int lid = xcd_chunk(blockIdx.x, gridDim.x);
  const int pair = lid % npair, split = lid / npair;
  const int cb = pair % n_co, kb = pair / n_co;
  const int c0 = cb * C::BCO, k0 = kb * C::BCI;
  const int t_begin = (int)((long long)split * n_tiles / splits);
  const int t_end = (int)((long long)(split + 1) * n_tiles / splits);

  const unsigned long long gbytes =
      ((unsigned long long)p.n * p.oh * p.ow - 1) * (unsigned long long)p.g_ld * 2ull + (unsigned long long)p.cout * 2ull;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.g + (size_t)c0 * 2), 0, (int)(gbytes - (unsigned long long)c0 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.x + (size_t)k0 * 2), 0, (int)(xbytes - (unsigned long long)k0 * 2), 0x00020000);
  const unsigned grow = (unsigned)p.g_ld * 2u, xrow = (unsigned)p.x_ld * 2u;

  // DMA lane geometry: a piece is 8 pixels x 128 B; lane -> pixel (lane>>3) of the piece and
  // LDS chunk (lane & 7), holding source chunk (lane & 7) ^ swz(row).  Rows of 8 pixels start
  // at multiples of 8, so swz(row) = 4 * ((row >> 1) & 1) depends on the lane only.
  const int lrow = lane >> 3, lch = lane & 7;
  const int lcs = lch ^ (((lrow >> 1) & 1) << 2);

  struct TilePos {
    int n, y0, x0, col, ty, tx;
  };
  auto tpos = [&](int t) {  // (divisions: once per workgroup)
    TilePos q;
    q.ty = t % tiles_y;
    q.col = t / tiles_y;
    q.tx = q.col % tiles_x;
    q.n = q.col / tiles_x;
    q.x0 = q.tx * 64;
    q.y0 = q.ty * PR;
    return q;
  };
  auto tnext = [&](TilePos q) {  // tile t + 1 from tile t (scalar increments, no divisions)
    if (++q.ty == tiles_y) {
      q.ty = 0;
      ++q.col;
      if (++q.tx == tiles_x) {
        q.tx = 0;
        ++q.n;
      }
    }
    q.x0 = q.tx * 64;
    q.y0 = q.ty * PR;
    return q;
  };

  // G tile of tile T into G buffer gb.  Per-lane parts (row in the tile, channel chunk) once;
  // per tile one wave-uniform base and two range limits.
  constexpr int GQ = (TMO * C::GPI + NW - 1) / NW;
  unsigned gofs[GQ];
  int grd[GQ], grm[GQ];
  bool gok[GQ];
#pragma unroll
  for (int q = 0; q < GQ; ++q) {
    const int pc = wave + NW * q;
    const int sub = pc / C::GPI, pr = pc - sub * C::GPI;
    const int row = pr * 8 + lrow;
    const int ch = 64 * sub + lcs * 8;
    grd[q] = row / 64;
    grm[q] = row & 63;
    gok[q] = pc < TMO * C::GPI && c0 + ch < p.cout;
    gofs[q] = (unsigned)(grd[q] * p.ow + grm[q]) * grow + (unsigned)ch * 2u;
  }
  auto issue_g = [&](const TilePos& T, int gb) {
    char* G = smem + gb * C::GSZ;
    const unsigned base = (unsigned)((T.n * p.oh + T.y0) * p.ow + T.x0) * grow;
    const int ylim = p.oh - T.y0, xlim = p.ow - T.x0;
#pragma unroll
    for (int q = 0; q < GQ; ++q) {
      const int pc = wave + NW * q;
      if (pc < TMO * C::GPI) {
        const unsigned o = (gok[q] && grd[q] < ylim && grm[q] < xlim) ? base + gofs[q] : OOB;
        lds_dma16(rg, G + pc * 1024, o);
      }
    }
  };
  // halo rows [h0, h0 + NR) (relative to tile T's first halo row) into their ring slots
  // (nr: std::integral_constant<int, NR>, so the piece -> row divisions are by constants)
  auto issue_x = [&](const TilePos& T, int h0, auto nr) {
    constexpr int npc = decltype(nr)::value * C::XPR;  // pieces per sub-image
#pragma unroll 1
    for (int pc = wave; pc < TMI * npc; pc += NW) {
      const int sub = pc / npc, rem = pc - sub * npc;
      const int hrow = h0 + rem / C::XPR, piece = rem - (rem / C::XPR) * C::XPR;
      const int hx = piece * 8 + lrow;
      const int iy = T.y0 + p.dy0 + hrow, ix = T.x0 + p.dx0 + hx;
      const int slot = (T.y0 + hrow) % C::R;
      const int ch = 64 * sub + lcs * 8;
      const bool ok = hx < 64 + TW - 1 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw && k0 + ch < p.c;
      const unsigned o = ok ? (unsigned)((T.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)ch * 2u : OOB;
      char* dst = smem + 2 * C::GSZ + sub * C::XSUB + (slot * C::XW + piece * 8) * 128;
      lds_dma16(rx, dst, o);
    }
  };

  // The steady-state refill (a tile's PR new halo rows, same column): per-lane column and
  // channel parts once, per tile one wave-uniform base; the piece -> (row, column block) split
  // is uniform per piece index (no per-issue divisions).
  constexpr int XNP = PR * C::XPR;                          // pieces per sub-image
  constexpr int XQ = (TMI * XNP + NW - 1) / NW;             // pieces per wave
  unsigned xofs[XQ];
  int xhx[XQ];
  bool xok[XQ];
#pragma unroll
  for (int q = 0; q < XQ; ++q) {
    const int pc = wave + NW * q;
    const int sub = pc / XNP, rem = pc - sub * XNP;
    const int hr = rem / C::XPR, piece = rem - hr * C::XPR;
    const int hx = piece * 8 + lrow;
    const int ch = 64 * sub + lcs * 8;
    xhx[q] = hx;
    xok[q] = pc < TMI * XNP && hx < 64 + TW - 1 && k0 + ch < p.c;
    xofs[q] = (unsigned)(hr * p.iw + hx) * xrow + (unsigned)ch * 2u;
  }
  auto issue_x_new = [&](const TilePos& T) {
    const int h0 = C::HR - PR;
    const int yb = T.y0 + p.dy0 + h0, xb = T.x0 + p.dx0;
    const long long base = ((long long)(T.n * p.ih + yb) * p.iw + xb) * (long long)xrow;
    int ys = (T.y0 + h0) % C::R;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= TMI * XNP) continue;  // (wave-uniform)
      const int sub = pc / XNP, rem = pc - sub * XNP;
      const int hr = rem / C::XPR, piece = rem - hr * C::XPR;  // (constants per unrolled q and wave)
      int slot = ys + hr;
      slot -= slot >= C::R ? C::R : 0;
      const bool rowok = (unsigned)(yb + hr) < (unsigned)p.ih;
      const bool ok = xok[q] && rowok && (unsigned)(xb + xhx[q]) < (unsigned)p.iw;
      const unsigned o = ok ? (unsigned)(base + (long long)xofs[q]) : OOB;
      char* dst = smem + 2 * C::GSZ + sub * C::XSUB + (slot * C::XW + piece * 8) * 128;
      lds_dma16(rx, dst, o);
    }
  };

  // transposed-read lane addressing: lane 4q+p of 16-lane group grp reads row (4u + q) of the
  // group's 4-row block and 8 bytes at column 16*(grp&1) + 4p of the operand's 32 columns
  const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  auto tr_off = [&](int col0, int m) {
    const int row = m + tq;
    const int col = col0 + 16 * (grp & 1) + 4 * tp;
    const int ch = (col >> 3) ^ (((row >> 1) & 1) << 2);
    return row * 128 + ch * 16 + (col & 7) * 2 + 8 * 128 * (grp >> 1);
  };

  f32x16 acc[C::NACC];
#pragma unroll
  for (int a = 0; a < C::NACC; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[a][e] = 0.f;

  const int wco = NW == 8 ? (wave >> 1) & 1 : 0, wci = wave & 1, wrow = NW == 8 ? wave >> 2 : wave >> 1;
  // bias gradient (p.bws): the ci-block-0 workgroups' wci = 0 waves sum the G fragments they
  // already hold for the MFMAs (lane l: co = l % 32 of the fragment, 8 pixels)
  const bool dob = DOB && p.bws != nullptr && kb == 0 && wci == 0;
  float bsum[TMO];
#pragma unroll
  for (int j = 0; j < TMO; ++j) bsum[j] = 0.f;
  int g_off[TMO], x_off[4][TMI];
#pragma unroll
  for (int j = 0; j < TMO; ++j) {
    const int col = wco * 32 * TMO + 32 * j;
    g_off[j] = (col >> 6) * C::GSUB + tr_off(col & 63, 0);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < TMI; ++j) {
      const int col = wci * 32 * TMI + 32 * j;
      x_off[m][j] = (col >> 6) * C::XSUB + tr_off(col & 63, m);
    }

  if (t_begin < t_end) {
    const TilePos T0 = tpos(t_begin);
    issue_g(T0, 0);
    issue_x(T0, 0, std::integral_constant<int, C::HR>());
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  int gb = 0;
  TilePos Tc = tpos(t_begin < t_end ? t_begin : 0);
  for (int tile = t_begin; tile < t_end; ++tile, gb ^= 1) {
    const TilePos T = Tc;
    const bool has_next = tile + 1 < t_end;
    const TilePos TN = has_next ? tnext(T) : T;
    Tc = TN;
    const bool same_col = has_next && TN.col == T.col;
    if (same_col && !(dbg & 8)) {  // next tile: its G tile and its PR new halo rows
      issue_g(TN, gb ^ 1);
      issue_x_new(TN);
    }
    const char* G = smem + gb * C::GSZ;
    const char* X = smem + 2 * C::GSZ;
    if constexpr (PIPE) {
      constexpr int NS = (PR / 2) * 4, NB = C::NT * TMI;
      // LDS bases of the halo rows this wave's k-steps read (rows wrow * PR/2 + j of the tile),
      // ring wrap resolved once per tile rather than per k-step and tap
      constexpr int NXR = PR / 2 + TH - 1;
      const char* Xrow[NXR];
      {
        int slot = (T.y0 + wrow * (PR / 2)) % C::R;
#pragma unroll
        for (int j = 0; j < NXR; ++j) {
          Xrow[j] = X + slot * (C::XW * 128);
          slot = slot + 1 == C::R ? 0 : slot + 1;
        }
      }
      bf16x8 pa[2][TMO], pb[2][NB];
      auto load = [&](int st, int k) {
        if ((dbg & 64) && st >= 2) return;
        const int py = wrow * (PR / 2) + (st >> 2), kx = st & 3;
        const int gr = py * 64 + kx * 16;
#pragma unroll
        for (int j = 0; j < TMO; ++j) pa[k][j] = tr_pair(G + g_off[j] + gr * 128, G + g_off[j] + gr * 128 + 4 * 128);
#pragma unroll
        for (int ti = 0; ti < TH; ++ti) {
          const char* Xr = Xrow[(st >> 2) + ti];
#pragma unroll
          for (int tj = 0; tj < TW; ++tj) {
            const int xr = kx * 16 + tj;
            const int m = xr & 3, xb = xr - m;
#pragma unroll
            for (int ji = 0; ji < TMI; ++ji)
              pb[k][(ti * TW + tj) * TMI + ji] =
                  tr_pair(Xr + x_off[m][ji] + xb * 128, Xr + x_off[m][ji] + xb * 128 + 4 * 128);
          }
        }
      };
      auto mma = [&](int k) {
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
          for (int ji = 0; ji < TMI; ++ji)
#pragma unroll
            for (int jo = 0; jo < TMO; ++jo) {
              f32x16& c = acc[(t * TMO + jo) * TMI + ji];
              const bf16x8 b = pb[k][t * TMI + ji];
              if (dbg & 16)
                c[0] += __builtin_bit_cast(float, __builtin_bit_cast(i32x4, pa[k][jo])[0] ^ __builtin_bit_cast(i32x4, b)[1]);
              else
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[k][jo], b, c, 0, 0, 0);
            }
        if constexpr (DOB) {
#pragma unroll
          for (int j = 0; j < TMO; ++j) bsum[j] = sum8_bf16(pa[k][j], bsum[j]);
        }
      };
      load(0, 0);
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        if (st + 1 < NS) load(st + 1, (st + 1) & 1);
        mma(st & 1);
        if (st + 1 < NS) {  // each MFMA followed by two of the next step's transposed reads
#pragma unroll
          for (int i = 0; i < NB * TMO; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // the next step's reads stay in this step
      }
    } else
#pragma unroll
    for (int pyl = 0; pyl < PR / 2; ++pyl)
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        const int py = wrow * (PR / 2) + pyl;
        const int gr = py * 64 + kx * 16;  // first G row of this k-step (multiple of 16)
        bf16x8 a[TMO];
#pragma unroll
        for (int j = 0; j < TMO; ++j) a[j] = tr_pair(G + g_off[j] + gr * 128, G + g_off[j] + gr * 128 + 4 * 128);
#pragma unroll
        for (int ti = 0; ti < TH; ++ti) {
          const int slot = (T.y0 + py + ti) % C::R;  // ring slot of halo row py + ti (uniform)
          const char* Xr = X + slot * (C::XW * 128);
#pragma unroll
          for (int tj = 0; tj < TW; ++tj) {
            const int t = ti * TW + tj;
            const int xr = kx * 16 + tj;  // first pixel of the k-step in the halo row
            const int m = xr & 3, xb = xr - m;
#pragma unroll
            for (int ji = 0; ji < TMI; ++ji) {
              const bf16x8 b = tr_pair(Xr + x_off[m][ji] + xb * 128, Xr + x_off[m][ji] + xb * 128 + 4 * 128);
#pragma unroll
              for (int jo = 0; jo < TMO; ++jo) {
                f32x16& c = acc[(t * TMO + jo) * TMI + ji];
                if (dbg & 16)
                  c[0] += __builtin_bit_cast(float, __builtin_bit_cast(i32x4, a[jo])[0] ^ __builtin_bit_cast(i32x4, b)[1]);
                else
                  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[jo], b, c, 0, 0, 0);
              }
            }
          }
        }
        // every wave sums (4 VALU per fragment, no branch to split the k-step's schedule);
        // only the dob waves write the result
#pragma unroll
        for (int j = 0; j < TMO; ++j) bsum[j] = sum8_bf16(a[j], bsum[j]);
      }
    if (!(dbg & 128)) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    if (has_next && !same_col) {  // column change: refill the whole ring (pipeline restart)
      issue_g(TN, gb ^ 1);
      issue_x(TN, 0, std::integral_constant<int, C::HR>());
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  }

  // bias partials: lanes l and l + 32 hold the two 8-pixel halves of the same channel;
  // the two row halves write separate slabs (2 * split + wrow)
  if (dob) {
#pragma unroll
    for (int j = 0; j < TMO; ++j) {
      const float t = bsum[j] + __shfl_xor(bsum[j], 32, 64);
      const int co = c0 + wco * 32 * TMO + 32 * j + (lane & 31);
      if (lane < 32 && co < p.cout) p.bws[(long long)(2 * split + wrow) * p.cout + co] = t;
    }
  }

  // ---- partial slab ws[split][co][t*c + ci] ----
  // The two row halves are summed through LDS first (one slab per split: half the slab
  // writes and half the reduction's reads).  Each row half owns half the taps: a wave parks
  // the taps its partner owns (lane-fastest, conflict-free), one barrier, and adds the parked
  // values to its own taps as it stores them -- both halves store, behind a single barrier.
  // C layout: column (ci) = lane & 31, rows (co) = 8*(e>>2) + 4*(lane>>5) + (e&3)
  // slab rows: NT * c values, or ws_taps * c of which this launch fills its taps' column
  // blocks (p.tmap; the stride-2 weight gradient's four phase launches share one slab set)
  const long long ws_k = (long long)(p.ws_taps > 0 ? p.ws_taps : C::NT) * p.c;
  const int r32 = lane & 31, hh = lane >> 5;
  float* slab = p.ws + (long long)(merge ? split : 2 * split + wrow) * p.cout * ws_k;
  constexpr int TO = (C::NT + 1) / 2;  // taps [0, TO) are row half 0's, [TO, NT) row half 1's
  constexpr int PSZ = TMO * TMI * 16 * 64;  // floats per parked tap of one wave
  static_assert((NW / 2) * C::NT * PSZ * 4 <= C::SMEM, "row-half exchange fits the LDS");
  float* X = (float*)smem + (wco * 2 + wci) * (C::NT * PSZ) + lane;
  if (merge) {
#pragma unroll
    for (int t = 0; t < C::NT; ++t)
      if ((t < TO) != (wrow == 0)) {
#pragma unroll
        for (int j = 0; j < TMO * TMI; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) X[t * PSZ + (j * 16 + e) * 64] = acc[t * TMO * TMI + j][e];
      }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < C::NT; ++t) {
    if (merge && (t < TO) != (wrow == 0)) continue;
#pragma unroll
    for (int jo = 0; jo < TMO; ++jo)
#pragma unroll
      for (int ji = 0; ji < TMI; ++ji) {
        const int ci = k0 + wci * 32 * TMI + 32 * ji + r32;
        if (ci >= p.c) continue;
        const int j = jo * TMI + ji;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = c0 + wco * 32 * TMO + 32 * jo + 8 * (e >> 2) + 4 * hh + (e & 3);
          if (co < p.cout && (!(dbg & 32) || acc[t * TMO * TMI + j][e] == 12345.678f))
            slab[(long long)co * ws_k + (long long)(p.ws_taps > 0 ? (p.tmap >> (4 * t)) & 15 : t) * p.c + ci] =
                acc[t * TMO * TMI + j][e] + (merge ? X[t * PSZ + (j * 16 + e) * 64] : 0.f);
        }
      }
  }
}

// 1x1 weight gradient of two wide layers (c, cout > 128; the 448 -> 448 HRNet heads): a
// workgroup owns a 256 x 256 (co x ci) block, so each 64-pixel tile's G and X images (32 KB
// each) feed 4x the MFMAs of the 128 x 128 block (half the L2 -> CU bytes per MFMA: the
// 128-block kernel sat at the CU's fetch rate).  1x1 stride-1 unpadded: the pixels are one
// flat range, a tile is 64 consecutive pixels.  8 waves = 2 (co) x 4 (ci), a wave owns
// 128 co x 64 ci (4 x 2 accumulators); G and X are double-buffered (128 KB), one barrier per
// tile.  One partial slab per split, summed by dvie_wgrad_reduce.
template <bool DOB>
__device__ __forceinline__ void wgrad_wide_body(const dvie_wgrad_desc& p, char* smem, int c0, int k0, int split, int t_begin,
                                                int t_end) {
  constexpr int NW = 8, NSUB = 4, SUB = 64 * 128, TSZ = NSUB * SUB, PQ = NSUB * 8 / NW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned OOB = 0xFFFFFFF0u;
  const long long npix = (long long)p.n * p.oh * p.ow;
  const unsigned long long gbytes = ((unsigned long long)npix - 1) * (unsigned long long)p.g_ld * 2ull + (unsigned long long)p.cout * 2ull;
  const unsigned long long xbytes = ((unsigned long long)npix - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.g + (size_t)c0 * 2), 0, (int)(gbytes - (unsigned long long)c0 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.x + (size_t)k0 * 2), 0, (int)(xbytes - (unsigned long long)k0 * 2), 0x00020000);
  const unsigned grow = (unsigned)p.g_ld * 2u, xrow = (unsigned)p.x_ld * 2u;
  // DMA lane geometry as in wgrad_halo_kernel (piece = 8 pixels x 128 B); the per-lane parts
  // of the offsets once, per tile one wave-uniform base and a pixel limit
  const int lrow = lane >> 3, lch = lane & 7;
  const int lcs = lch ^ (((lrow >> 1) & 1) << 2);
  int ppx[PQ];
  unsigned goff[PQ], xoff[PQ];
  bool gok[PQ], xok[PQ];
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const int pc = wave + NW * q, sub = pc >> 3, pr = pc & 7;
    const int ch = 64 * sub + lcs * 8;
    ppx[q] = pr * 8 + lrow;
    goff[q] = (unsigned)ppx[q] * grow + (unsigned)ch * 2u;
    xoff[q] = (unsigned)ppx[q] * xrow + (unsigned)ch * 2u;
    gok[q] = c0 + ch < p.cout;
    xok[q] = k0 + ch < p.c;
  }
  auto issue = [&](int tile, int buf) {
    const int P0 = tile * 64;
    const int lim = (int)min((long long)64, npix - (long long)P0);
    const unsigned bg = (unsigned)P0 * grow, bx = (unsigned)P0 * xrow;
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int pc = wave + NW * q, sub = pc >> 3, pr = pc & 7;
      const bool in = ppx[q] < lim;
      lds_dma16(rg, smem + buf * TSZ + sub * SUB + pr * 1024, (in && gok[q]) ? bg + goff[q] : OOB);
      lds_dma16(rx, smem + (2 + buf) * TSZ + sub * SUB + pr * 1024, (in && xok[q]) ? bx + xoff[q] : OOB);
    }
  };
  const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  auto tr_off = [&](int col0) {
    const int col = col0 + 16 * (grp & 1) + 4 * tp;
    const int ch = (col >> 3) ^ (((tq >> 1) & 1) << 2);
    return tq * 128 + ch * 16 + (col & 7) * 2 + 8 * 128 * (grp >> 1);
  };
  const int wco = wave >> 2, wci = wave & 3;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  int g_off[4], x_off[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wco * 128 + 32 * j;
    g_off[j] = (col >> 6) * SUB + tr_off(col & 63);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int col = wci * 64 + 32 * i;
    x_off[i] = (col >> 6) * SUB + tr_off(col & 63);
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;
  if (t_begin < t_end) {
    issue(t_begin, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  int buf = 0;
  for (int tile = t_begin; tile < t_end; ++tile, buf ^= 1) {
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    const char* G = smem + buf * TSZ;
    const char* X = smem + (2 + buf) * TSZ;
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) {
      const int r = kx * 16 * 128;
      bf16x8 a[4], b[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = tr_pair(G + g_off[j] + r, G + g_off[j] + r + 4 * 128);
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = tr_pair(X + x_off[i] + r, X + x_off[i] + r + 4 * 128);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j], b[i], acc[j][i], 0, 0, 0);
      if constexpr (DOB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bsum[j] = sum8_bf16(a[j], bsum[j]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  if constexpr (DOB) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = bsum[j] + __shfl_xor(bsum[j], 32, 64);
      const int co = c0 + wco * 128 + 32 * j + (lane & 31);
      if (lane < 32 && co < p.cout) p.bws[(long long)split * p.cout + co] = t;
    }
  }
  // partial slab ws[split][co][ci]; C layout: column (ci) = lane & 31, rows (co) =
  // 8*(e>>2) + 4*(lane>>5) + (e&3)
  const int r32 = lane & 31, hh = lane >> 5;
  float* slab = p.ws + (long long)split * p.cout * p.c;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = k0 + wci * 64 + 32 * i + r32;
      if (ci >= p.c) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = c0 + wco * 128 + 32 * j + 8 * (e >> 2) + 4 * hh + (e & 3);
        if (co < p.cout) slab[(long long)co * p.c + ci] = acc[j][i][e];
      }
    }
}

__global__ __launch_bounds__(512) void wgrad_wide_kernel(const dvie_wgrad_desc p, int n_co, int n_ci, int splits,
                                                         int n_tiles) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * 4 * 64 * 128];
  const int npair = n_co * n_ci;
  const int lid = xcd_chunk(blockIdx.x, gridDim.x);
  const int pair = lid % npair, split = lid / npair;
  const int c0 = (pair % n_co) * 256, k0 = (pair / n_co) * 256;
  const int t_begin = (int)((long long)split * n_tiles / splits);
  const int t_end = (int)((long long)(split + 1) * n_tiles / splits);
  // bias column sums (the ci-block-0 workgroups' wci = 0 waves, from the G fragments they hold
  // for the MFMAs): compiled as its own body, so the other waves and workgroups carry none of
  // the summing (a wave-uniform choice, made once)
  const int wci = (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) & 3;
  if (p.bws != nullptr && k0 == 0 && wci == 0)
    wgrad_wide_body<true>(p, smem, c0, k0, split, t_begin, t_end);
  else
    wgrad_wide_body<false>(p, smem, c0, k0, split, t_begin, t_end);
}

// diagnostic override, read once (plan-time slab counts and launches must agree):
// DVIE_WGRAD_HALO=0 = per-tap kernel only
static const bool wg_halo_env_off = getenv("DVIE_WGRAD_HALO") && *getenv("DVIE_WGRAD_HALO") == '0';

static bool wgrad_halo_eligible(const dvie_wgrad_desc& p) {
  if (p.dtype != DVIE_BF16) return false;
  if (wg_halo_env_off) return false;
  if (p.sy != 1 || p.sx != 1 || p.ddy != 1 || p.ddx != 1) return false;
  if (!((p.th == 1 && p.tw == 1) || (p.th == 3 && p.tw == 3) || (p.th <= 2 && p.tw <= 2))) return false;
  if (p.ws_taps > 0 && (p.ws_taps > 16 || p.th * p.tw > 4)) return false;
  if (p.c % 8 != 0 || p.cout % 8 != 0) return false;
  if (p.g_ld % 8 != 0 || p.x_ld % 8 != 0) return false;
  const unsigned long long npx = (unsigned long long)p.n * p.ih * p.iw, npg = (unsigned long long)p.n * p.oh * p.ow;
  if (npx >= (1ull << 31) || npg >= (1ull << 31)) return false;
  // the kernel forms 32-bit buffer offsets: both operands' byte spans must fit (else the
  // per-tap kernel, 64-bit addressing, takes the launch)
  const unsigned long long xspan = ((npx - 1) * (unsigned long long)p.x_ld + (unsigned long long)p.c) * 2ull;
  const unsigned long long gspan = ((npg - 1) * (unsigned long long)p.g_ld + (unsigned long long)p.cout) * 2ull;
  if (xspan >= 0xFFFFFF00ull || gspan >= 0xFFFFFF00ull) return false;
  return true;
}

struct WgPlan {
  int pr, tmo, tmi, wide;
};

// DVIE_WG_NARROW=0: 3x3 layers with <= 32 output channels on the 8-wave kernel (A/B runs)
static const bool wg_narrow_env_off = getenv("DVIE_WG_NARROW") && *getenv("DVIE_WG_NARROW") == '0';

// DVIE_WG_WIDE=0: 1x1 wide layers on the 128 x 128 block kernel (A/B runs)
static const bool wg_wide_env_off = getenv("DVIE_WG_WIDE") && *getenv("DVIE_WG_WIDE") == '0';

static WgPlan wgrad_plan(const dvie_wgrad_desc& p) {
  // (the phase launches of one shared slab set all take this plan: equal tiles and splits)
  if (p.th > 1 || p.tw > 1 || p.ws_taps > 0) return {4, 1, 1, 0};
  if (!wg_wide_env_off && p.ws_taps == 0 && p.c > 128 && p.cout > 128 && p.dy0 == 0 && p.dx0 == 0 && p.oh == p.ih && p.ow == p.iw)
    return {1, 4, 4, 1};
  const char* e = getenv("DVIE_WG_TM");  // tuning override for 1x1: "<tmo><tmi>", e.g. "11"
  if (e && e[0] && e[1]) return {2, e[0] == '2' ? 2 : 1, e[1] == '2' ? 2 : 1, 0};
  return {2, p.cout > 64 ? 2 : 1, p.c > 64 ? 2 : 1, 0};
}

static void wgrad_tiles(const dvie_wgrad_desc& p, const WgPlan& w, int& tiles_x, int& tiles_y, int& n_tiles, int& n_co,
                        int& n_ci) {
  if (w.wide) {  // flat 64-pixel tiles, 256-channel blocks
    tiles_x = tiles_y = 1;
    n_tiles = (int)(((long long)p.n * p.oh * p.ow + 63) / 64);
    n_co = (p.cout + 255) / 256;
    n_ci = (p.c + 255) / 256;
    return;
  }
  tiles_x = (p.ow + 63) / 64;
  tiles_y = (p.oh + w.pr - 1) / w.pr;
  n_tiles = tiles_x * tiles_y * p.n;
  n_co = (p.cout + 64 * w.tmo - 1) / (64 * w.tmo);
  n_ci = (p.c + 64 * w.tmi - 1) / (64 * w.tmi);
}

// splits the halo kernel wants (0: not eligible -> the per-tap kernel with caller's splits)
int wgrad_halo_splits(const dvie_wgrad_desc& p) {
  if (!wgrad_halo_eligible(p)) return 0;
  const WgPlan w = wgrad_plan(p);
  int tx, ty, nt, nco, nci;
  wgrad_tiles(p, w, tx, ty, nt, nco, nci);
  int s = 256 / (nco * nci);  // one workgroup per CU (LDS-bound): a single wave of workgroups
  const char* e = getenv("DVIE_WG_SPLITS");  // tuning: multiplier of that split count (e.g. 0.5)
  if (e && *e && atof(e) > 0) s = (int)(s * atof(e) + 0.5);
  if (s > nt) s = nt;
  return s < 1 ? 1 : s;
}

// one partial slab per split (the kernel sums its two row halves)
// DVIE_WG_MERGE=0: two slabs per split, row halves unmerged (A/B runs)
static const int wg_merge = getenv("DVIE_WG_MERGE") && *getenv("DVIE_WG_MERGE") == '0' ? 0 : 1;
// timing-only ablation bits (DVIE_WG_DBG, -DDVIE_TIMING_DBG builds; read per launch)
static int wg_dbg() {
#ifdef DVIE_TIMING_DBG
  const char* e = getenv("DVIE_WG_DBG");
  return e && *e ? atoi(e) : 0;
#else
  return 0;
#endif
}
// DVIE_SETPRIO=1: s_setprio 1 for the second half of the waves in the halo conv / weight-gradient
// kernels (A/B runs)
static const int wg_setprio = getenv("DVIE_SETPRIO") && *getenv("DVIE_SETPRIO") == '1' ? 2 : 0;

// DVIE_WG_PIPE (A/B, read per launch): 0 = 3x3 weight gradients without the fragment pipeline
static bool wg_pipe_on() {
  const char* e = getenv("DVIE_WG_PIPE");
  return !(e && *e == '0');
}

// bias partial slabs the halo kernels write to p.bws (0: the launch is not theirs)
int wgrad_halo_bias_slabs(const dvie_wgrad_desc& p) {
  if (!wgrad_halo_eligible(p)) return 0;
  return wgrad_plan(p).wide ? p.splits : 2 * p.splits;
}

int wgrad_halo_slabs(const dvie_wgrad_desc& p) {
  return wgrad_halo_eligible(p) && !wg_merge && !wgrad_plan(p).wide ? 2 * p.splits : p.splits;
}

bool wgrad_halo_launch(const dvie_wgrad_desc& p, hipStream_t s) {
  if (!wgrad_halo_eligible(p)) return false;
  const WgPlan w = wgrad_plan(p);
  int tiles_x, tiles_y, n_tiles, n_co, n_ci;
  wgrad_tiles(p, w, tiles_x, tiles_y, n_tiles, n_co, n_ci);
  const int grid = n_co * n_ci * p.splits;
  const bool wg_pipe = wg_pipe_on();
  if (w.wide) {
    DVIE_LAUNCH(wgrad_wide_kernel, dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits, n_tiles);
    return true;
  }
#define DVIE_WG(TH, PR, TMO, TMI)                                                                                   \
  DVIE_LAUNCH((wgrad_halo_kernel<TH, TH, PR, TMO, TMI>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits, \
                     tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio)
#ifdef DVIE_TIMING_DBG
  if (p.th == 3 && p.cout > 32 && wg_pipe && wg_dbg()) {
    switch (wg_dbg()) {
#define DVIE_WG_AB(V)                                                                                             \
  case V:                                                                                                         \
    DVIE_LAUNCH((wgrad_halo_kernel<3, 3, 4, 1, 1, 8, true, V>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits, \
                tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);                                                 \
    return true;
      DVIE_WG_AB(8) DVIE_WG_AB(16) DVIE_WG_AB(32) DVIE_WG_AB(64) DVIE_WG_AB(128) DVIE_WG_AB(136) DVIE_WG_AB(80)
      DVIE_WG_AB(192) DVIE_WG_AB(144)
#undef DVIE_WG_AB
      default: break;
    }
  }
#endif
  if (p.th == 3 && p.cout > 32 && wg_pipe && !p.bws)
    DVIE_LAUNCH((wgrad_halo_kernel<3, 3, 4, 1, 1, 8, true, 0, false>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci,
                p.splits, tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
  else if (p.th == 3 && p.cout > 32 && wg_pipe)
    DVIE_LAUNCH((wgrad_halo_kernel<3, 3, 4, 1, 1, 8, true>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits,
                       tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
  // the stride-2 weight gradient's phase launches (ws_taps): 2 x 2, 2 x 1, 1 x 2 tap grids
#define DVIE_WG2(TH, TW)                                                                                        \
  else if (p.th == TH && p.tw == TW && !p.bws)                                                                  \
    DVIE_LAUNCH((wgrad_halo_kernel<TH, TW, 4, 1, 1, 8, true, 0, false>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, \
                p.splits, tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);                                        \
  else if (p.th == TH && p.tw == TW)                                                                            \
    DVIE_LAUNCH((wgrad_halo_kernel<TH, TW, 4, 1, 1, 8, true>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits, \
                tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
  DVIE_WG2(2, 2) DVIE_WG2(2, 1) DVIE_WG2(1, 2)
  else if (p.ws_taps > 0 && p.th == 1 && p.tw == 1 && !p.bws)
    DVIE_LAUNCH((wgrad_halo_kernel<1, 1, 4, 1, 1, 8, true, 0, false>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci,
                p.splits, tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
  else if (p.ws_taps > 0 && p.th == 1 && p.tw == 1)
    DVIE_LAUNCH((wgrad_halo_kernel<1, 1, 4, 1, 1, 8, true>), dim3(grid), dim3(512), 0, s, p, n_co, n_ci, p.splits,
                tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
#undef DVIE_WG2
  else if (p.th == 3 && p.cout <= 32 && !wg_narrow_env_off)
    DVIE_LAUNCH((wgrad_halo_kernel<3, 3, 4, 1, 1, 4, true>), dim3(grid), dim3(256), 0, s, p, n_co, n_ci, p.splits,
                       tiles_x, tiles_y, n_tiles, wg_merge | wg_setprio);
  else if (p.th == 3)
    DVIE_WG(3, 4, 1, 1);
  else if (w.tmo == 2 && w.tmi == 2)
    DVIE_WG(1, 2, 2, 2);
  else if (w.tmo == 2)
    DVIE_WG(1, 2, 2, 1);
  else if (w.tmi == 2)
    DVIE_WG(1, 2, 1, 2);
  else
    DVIE_WG(1, 2, 1, 1);
#undef DVIE_WG
  return true;
}

}  // namespace dvie
