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

template <int TH, int TW, int PR, int TMO, int TMI>
struct WgCfg {
  static constexpr int NT = TH * TW;
  static constexpr int BCO = 64 * TMO, BCI = 64 * TMI;  // output / input channels per block
  static constexpr int HR = PR + TH - 1, HWD = 64 + TW - 1;
  static constexpr int GROWS = PR * 64;
  static constexpr int XROWS = HR * HWD;
  static constexpr int GPI = GROWS / 8;               // DMA pieces (8 rows x 128 B) per sub-image
  static constexpr int XPI = (XROWS + 7) / 8;
  static constexpr int GSUB = GPI * 1024, XSUB = XPI * 1024;  // one 64-channel sub-image
  static constexpr int GSZ = TMO * GSUB, XSZ = TMI * XSUB;
  static constexpr int NGP = TMO * GPI, NXP = TMI * XPI;
  static constexpr int GQ = (NGP + 3) / 4, XQ = (NXP + 3) / 4;
  static constexpr int BUF = GSZ + XSZ;
  static constexpr int SMEM = 2 * BUF;
  static constexpr int NACC = NT * TMO * TMI;
};

template <int TH, int TW, int PR, int TMO, int TMI>
__global__ __launch_bounds__(256) void wgrad_halo_kernel(const dvie_wgrad_desc p, int n_co, int n_ci, int splits,
                                                         int tiles_x, int tiles_y, int n_tiles) {
  typedef WgCfg<TH, TW, PR, TMO, TMI> C;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned OOB = 0xFFFFFFF0u;

  // block -> (co block, ci block, split); co/ci blocks fastest so that concurrently running
  // blocks share their g / x tiles in L2
  const int npair = n_co * n_ci;
  const int pair = blockIdx.x % npair, split = blockIdx.x / npair;
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

  // DMA lane geometry: piece q of a sub-image fills rows 8q .. 8q+7; lane -> row 8q + (lane>>3),
  // LDS chunk (lane & 7) holding source chunk (lane & 7) ^ swz(row).  Channels past cout / c
  // (padding of narrow layers) read as zeros.
  const int lrow = lane >> 3, lch = lane & 7;

  auto issue = [&](int tile, int buf) {
    const int tx = tile % tiles_x;
    const int t2 = tile / tiles_x;
    const int ty = t2 % tiles_y, n = t2 / tiles_y;
    const int y0 = ty * PR, x0 = tx * 64;
    char* G = smem + buf * C::BUF;
    char* X = G + C::GSZ;
#pragma unroll
    for (int q = 0; q < C::GQ; ++q) {
      const int pc = wave + 4 * q;  // piece over all sub-images
      if (pc < C::NGP) {
        const int sub = pc / C::GPI, pr = pc - sub * C::GPI;
        const int row = pr * 8 + lrow;
        const int oy = y0 + row / 64, ox = x0 + (row & 63);
        const int cs = lch ^ (((row >> 1) & 1) << 2);
        const int ch = 64 * sub + cs * 8;
        const unsigned o = (oy < p.oh && ox < p.ow && c0 + ch < p.cout)
                               ? (unsigned)((n * p.oh + oy) * p.ow + ox) * grow + (unsigned)ch * 2u
                               : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (lds_ptr_wg)(G + pc * 1024), 16, o, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < C::XQ; ++q) {
      const int pc = wave + 4 * q;
      if (pc < C::NXP) {
        const int sub = pc / C::XPI, pr = pc - sub * C::XPI;
        const int row = pr * 8 + lrow;
        const int hy = row / C::HWD, hx = row - (row / C::HWD) * C::HWD;
        const int iy = y0 + p.dy0 + hy, ix = x0 + p.dx0 + hx;
        const int cs = lch ^ (((row >> 1) & 1) << 2);
        const int ch = 64 * sub + cs * 8;
        const bool ok = row < C::XROWS && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw &&
                        k0 + ch < p.c;
        const unsigned o = ok ? (unsigned)((n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)ch * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_wg)(X + pc * 1024), 16, o, 0, 0, 0);
      }
    }
  };

  // transposed-read lane addressing: lane 4q+p of 16-lane group grp reads row (4u + q) of the
  // group's 4-row block and 8 bytes at column 16*(grp&1) + 4p of the operand's 32 columns
  const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  // byte offset inside a 64-channel sub-image for columns [col0, col0+32) and base row m (mod 4)
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

  // waves 2 x 2 over (co, ci): wave owns 32*TMO co x 32*TMI ci
  const int wco = wave >> 1, wci = wave & 1;
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
    issue(t_begin, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  int buf = 0;
  for (int tile = t_begin; tile < t_end; ++tile, buf ^= 1) {
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    const char* G = smem + buf * C::BUF;
    const char* X = G + C::GSZ;
#pragma unroll
    for (int py = 0; py < PR; ++py)
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        const int gr = py * 64 + kx * 16;  // first G row of this k-step (multiple of 16)
        bf16x8 a[TMO];
#pragma unroll
        for (int j = 0; j < TMO; ++j) a[j] = tr_pair(G + g_off[j] + gr * 128, G + g_off[j] + gr * 128 + 4 * 128);
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          const int ti = t / TW, tj = t % TW;
          const int xr = (py + ti) * C::HWD + kx * 16 + tj;  // first X row (any alignment)
          const int m = xr & 3, xb = xr - m;
#pragma unroll
          for (int ji = 0; ji < TMI; ++ji) {
            const bf16x8 b = tr_pair(X + x_off[m][ji] + xb * 128, X + x_off[m][ji] + xb * 128 + 4 * 128);
#pragma unroll
            for (int jo = 0; jo < TMO; ++jo) {
              f32x16& c = acc[(t * TMO + jo) * TMI + ji];
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[jo], b, c, 0, 0, 0);
            }
          }
        }
      }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- partial slab ws[split][co][t*c + ci] ----
  // C layout: column (ci) = lane & 31, rows (co) = 8*(e>>2) + 4*(lane>>5) + (e&3)
  const long long ws_k = (long long)C::NT * p.c;
  const int r32 = lane & 31, hh = lane >> 5;
  float* slab = p.ws + (long long)split * p.cout * ws_k;
#pragma unroll
  for (int t = 0; t < C::NT; ++t)
#pragma unroll
    for (int jo = 0; jo < TMO; ++jo)
#pragma unroll
      for (int ji = 0; ji < TMI; ++ji) {
        const int ci = k0 + wci * 32 * TMI + 32 * ji + r32;
        if (ci >= p.c) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = c0 + wco * 32 * TMO + 32 * jo + 8 * (e >> 2) + 4 * hh + (e & 3);
          if (co < p.cout) slab[(long long)co * ws_k + (long long)t * p.c + ci] = acc[(t * TMO + jo) * TMI + ji][e];
        }
      }
}

static bool wgrad_halo_eligible(const dvie_wgrad_desc& p) {
  if (p.dtype != DVIE_BF16) return false;
  if (p.sy != 1 || p.sx != 1 || p.ddy != 1 || p.ddx != 1) return false;
  if (!((p.th == 1 && p.tw == 1) || (p.th == 3 && p.tw == 3))) return false;
  if (p.c % 8 != 0 || p.cout % 8 != 0) return false;
  if (p.g_ld % 8 != 0 || p.x_ld % 8 != 0) return false;
  if ((unsigned long long)p.n * p.ih * p.iw >= (1ull << 31) || (unsigned long long)p.n * p.oh * p.ow >= (1ull << 31))
    return false;
  return true;
}

struct WgPlan {
  int pr, tmo, tmi;
};

static WgPlan wgrad_plan(const dvie_wgrad_desc& p) {
  if (p.th == 3) return {2, 1, 1};
  return {2, p.cout > 64 ? 2 : 1, p.c > 64 ? 2 : 1};
}

static void wgrad_tiles(const dvie_wgrad_desc& p, const WgPlan& w, int& tiles_x, int& tiles_y, int& n_tiles, int& n_co,
                        int& n_ci) {
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
  int s = (256 + nco * nci - 1) / (nco * nci);  // one workgroup per CU (LDS-bound), one wave of them
  if (s > nt) s = nt;
  return s < 1 ? 1 : s;
}

int wgrad_halo_slabs(const dvie_wgrad_desc& p) { return p.splits; }

bool wgrad_halo_launch(const dvie_wgrad_desc& p, hipStream_t s) {
  if (!wgrad_halo_eligible(p)) return false;
  const WgPlan w = wgrad_plan(p);
  int tiles_x, tiles_y, n_tiles, n_co, n_ci;
  wgrad_tiles(p, w, tiles_x, tiles_y, n_tiles, n_co, n_ci);
  const int grid = n_co * n_ci * p.splits;
#define DVIE_WG(TH, PR, TMO, TMI)                                                                                   \
  hipLaunchKernelGGL((wgrad_halo_kernel<TH, TH, PR, TMO, TMI>), dim3(grid), dim3(256), 0, s, p, n_co, n_ci, p.splits, \
                     tiles_x, tiles_y, n_tiles)
  if (p.th == 3)
    DVIE_WG(3, 2, 1, 1);
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
