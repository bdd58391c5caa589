// Narrow-output 3x3 convolution for gfx950, bf16: stride 1, at most 32 output channels,
// input channels a multiple of 32 and above 64 -- HRNet's 448 -> 3 / 448 -> 20 output heads
// (rgb_layer[2] / seg_layer[2], nets/HRNet.py:410-442 of the reference).
//
// Why a kernel of its own: on the chunked halo kernel (conv_halo.hip) these layers stream
// their whole weight tensor (32 x 4032 bf16, 258 KB) for every 4-row tile and run 8 MFMAs
// per wave between barriers (one (chunk, tap) step), so they are bound by step overhead and
// weight traffic, not by their 448-channel input.  Here one step is a 32-channel chunk with
// all nine taps: a workgroup of 8 waves owns an 8-row x 64-column output tile; per chunk it
// stages the input halo (10 x 66 pixels x 32 channels) and the chunk's weights for all taps
// (9 x 32 rows x 32 channels), both as 64-byte LDS rows whose four 16-B chunks are stored
// XOR-swizzled by bits 2-3 of the row (pixel) index, so the 16-lane groups of ds_read_b128
// hit distinct banks at any pixel shift and every DMA lane carries data (no pad slots); every
// wave then issues 36 MFMAs (9 taps x 2 k-slices x 2 pixel blocks) before the next barrier.
// Weight bytes per output pixel: 4032 x 64 B / 512 (vs / 256).
// Two stage buffers: chunk k+1 streams in (LDS-DMA) while chunk k computes; a workgroup
// walks an XCD-contiguous range of tiles, so the next tile's first chunk streams in under
// the current tile's last chunk and epilogue.
//
// MFMA v_mfma_f32_32x32x16_bf16: A = weights (32 output channels x 16 input channels),
// B = halo pixels (16 input channels x 32 pixels); epilogue from registers (permlane32
// pairing to 8 consecutive channels per lane) with bias / residual / accumulate /
// activation / activation-derivative, fp32 or bf16 output.
#include <stdlib.h>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_nr;

struct NarrowCfg {
  static constexpr int NW = 8;                          // waves = output rows per tile
  static constexpr int TW = 64;                         // output columns per tile
  static constexpr int HR = NW + 2, HW = TW + 2;        // halo rows / columns
  static constexpr int PITCH = 64;                      // LDS bytes per pixel / weight row
  static constexpr int HSLOTS = HR * HW * 4;            // 16-B slots of the halo image
  static constexpr int HPC = (HSLOTS + 63) / 64;        // its DMA pieces (1 KB each)
  static constexpr int WSLOTS = 9 * 32 * 4;             // weight image: [tap][co][32 ch]
  static constexpr int WPC = (WSLOTS + 63) / 64;
  static constexpr int PCS = HPC + WPC;                 // pieces per stage
  static constexpr int PPW = (PCS + NW - 1) / NW;       // per wave (upper bound)
  static constexpr int STAGE = PCS * 1024;
  static constexpr int SMEM = 2 * STAGE;
};
static_assert(NarrowCfg::SMEM <= 163840, "two stages fit the LDS");

__device__ __forceinline__ uint32_t pk2_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

__device__ __forceinline__ void narrow_act(float* v, int act, float alpha) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = act_bf(v[k], act, alpha);
}

template <bool OUTF32>
__global__ __launch_bounds__(512) void conv_narrow_kernel(const dvie_conv_desc p, int tiles_x, int tiles_y,
                                                          int n_tiles, int dbg) {
  dbg = DVIE_DBG(dbg);
  typedef NarrowCfg C;
  constexpr int NW = C::NW;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // XCD-contiguous tile range of this workgroup (blocks b and b + 8 share an XCD)
  const int G = gridDim.x;
  const int g = blockIdx.x & 7, i8 = blockIdx.x >> 3;
  const int nbg = G / 8 + (g < G % 8 ? 1 : 0);
  const int q8 = n_tiles / 8, rr = n_tiles % 8;
  const int t_begin = (g < rr ? g * (q8 + 1) : rr * (q8 + 1) + (g - rr) * q8) + i8;
  const int t_end = (g < rr ? g * (q8 + 1) : rr * (q8 + 1) + (g - rr) * q8) + q8 + (g < rr ? 1 : 0);
  if (t_begin >= t_end) return;
  const int my_tiles = (t_end - 1 - t_begin) / nbg + 1;
  const int nk = p.c >> 5;  // 32-channel chunks
  const int njobs = my_tiles * nk;

  // per-lane DMA geometry of this wave's pieces (tile- and chunk-independent)
  // halo piece: slot -> (row hy, column hx, source 16-B chunk cs); weight piece:
  // slot -> (tap t, channel co, cs)
  int geo[C::PPW];
#pragma unroll
  for (int q = 0; q < C::PPW; ++q) {
    const int pc = wave + NW * q;
    int v = -1;
    // lane -> stored chunk (slot & 3) of row slot >> 2, holding source chunk (slot & 3) ^ swz
    if (pc < C::HPC) {
      const int slot = pc * 64 + lane, px = slot >> 2, cs = (slot & 3) ^ ((px >> 2) & 3);
      if (px < C::HR * C::HW) v = ((px / C::HW) << 16) | ((px % C::HW) << 4) | cs;
    } else if (pc < C::PCS) {
      const int slot = (pc - C::HPC) * 64 + lane, row = slot >> 2, cs = (slot & 3) ^ ((row >> 2) & 3);
      if (row < 9 * 32 && (row & 31) < p.cout) v = (1 << 30) | ((row >> 5) << 16) | ((row & 31) << 4) | cs;
    }
    geo[q] = v;
  }
  const unsigned xrow = (unsigned)p.x_ld * 2u;
  const unsigned long long xbytes =
      ((unsigned long long)p.n * p.ih * p.iw - 1) * (unsigned long long)p.x_ld * 2ull + (unsigned long long)p.c * 2ull;
  const unsigned wbytes = (unsigned)p.cout * (unsigned)p.kpad * 2u;

  struct Tile {
    int n, y0, x0;
  };
  auto tile_of = [&](int i) {
    int t = t_begin + i * nbg;
    Tile T;
    T.x0 = (t % tiles_x) * C::TW;
    t /= tiles_x;
    T.y0 = (t % tiles_y) * NW;
    T.n = t / tiles_y;
    return T;
  };

  // job jj = (local tile jj / nk, chunk jj % nk) into stage buffer sb
  auto issue = [&](int jj, int sb) {
    if (dbg & 1) return;  // timing experiments only (DVIE_NARROW_DBG): no operand streaming
    const int k = jj % nk;
    const Tile T = tile_of(jj / nk);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.x + (size_t)k * 64), 0, (int)(xbytes - (unsigned long long)k * 64), 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.w + (size_t)k * 64), 0, (int)(wbytes - (unsigned)k * 64), 0x00020000);
    char* dst = smem + sb * C::STAGE;
    const int ybase = T.y0 + p.dy0, xbase = T.x0 + p.dx0;
#pragma unroll
    for (int q = 0; q < C::PPW; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::PCS) continue;  // (wave-uniform)
      const int v = geo[q];
      if (pc < C::HPC) {
        const int iy = ybase + ((v >> 16) & 0xFF), ix = xbase + ((v >> 4) & 0xFFF);
        const bool ok = v >= 0 && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw;
        const unsigned o = ok ? (unsigned)((T.n * p.ih + iy) * p.iw + ix) * xrow + (unsigned)(v & 15) * 16u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_nr)(dst + pc * 1024), 16, o, 0, 0, 0);
      } else {
        const int t = (v >> 16) & 0xF, co = (v >> 4) & 31;
        const unsigned o = v >= 0 ? (unsigned)(co * p.kpad + t * p.c) * 2u + (unsigned)(v & 15) * 16u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_nr)(dst + pc * 1024), 16, o, 0, 0, 0);
      }
    }
  };

  // fragment addresses within a stage: A (weights) row t*32 + r32, B (halo) pixel
  // (wave + ti, 32 b + tj + r32); k-slice s of the chunk = 16-B chunk 2 s + hh, stored at
  // (2 s + hh) ^ swz(row).  The weight rows' swizzle depends on r32 only; a pixel's on the
  // pixel index, i.e. on the tap shift.
  int a_off[2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) a_off[sl] = C::HPC * 1024 + r32 * C::PITCH + (((2 * sl + hh) ^ ((r32 >> 2) & 3)) << 4);
  const int px0 = wave * C::HW + r32;

  f32x16 acc[2];
  issue(0, 0);
  for (int jj = 0; jj < njobs; ++jj) {
    const int k = jj % nk;
    if (k == 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    }
    // job jj has landed for this wave (the only loads in flight), and for the others after
    // the barrier; every wave is also done reading the buffer job jj + 1 goes into
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
    if (jj + 1 < njobs) issue(jj + 1, (jj + 1) & 1);
    const char* S = smem + (jj & 1) * C::STAGE;
    if (dbg & 2) goto skip;  // timing experiments only: no MFMAs
    {
      // tap t + 1's fragments are read while tap t's MFMAs run (scheduling barriers keep the
      // compiler from interleaving each MFMA behind its own LDS round trip)
      i32x4 fa[2][2], fb[2][2][2];
      auto ld = [&](int t, int buf) {
        const int ti = t / 3, tj = t % 3;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          fa[buf][s] = *(const i32x4*)(S + a_off[s] + t * 32 * C::PITCH);
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int px = px0 + ti * C::HW + 32 * b + tj;
            const int boff = px * C::PITCH + ((hh ^ ((px >> 2) & 3)) << 4);  // k-slice s: xor 2s into the chunk
            fb[buf][s][b] = *(const i32x4*)(S + (boff ^ (s << 5)));
          }
        }
      };
      ld(0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[t & 1][s]),
                                                             __builtin_bit_cast(bf16x8, fb[t & 1][s][b]), acc[b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  skip:
    if (k + 1 < nk) continue;

    // ---- epilogue of the tile: lane owns pixel 32 b + r32 of row `wave`; after permlane32
    // pairing, lane half hh holds channels 16 P + 8 hh .. +7 of pair P
    const Tile T = tile_of(jj / nk);
    const int oy = T.y0 + wave;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float v[2][8];
#pragma unroll
      for (int P = 0; P < 2; ++P)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[b][8 * P + e]),
                                                           __float_as_uint(acc[b][8 * P + 4 + e]), false, false);
          v[P][e] = __uint_as_float(sw[0]);
          v[P][4 + e] = __uint_as_float(sw[1]);
        }
      const int ox = T.x0 + 32 * b + r32;
      if (oy >= p.oh || ox >= p.ow) continue;
      const long long pix = ((long long)T.n * p.oh + oy) * p.ow + ox;
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const int co = 16 * P + 8 * hh;
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
#pragma unroll
          for (int k = 0; k < 8; ++k) w[k] = act_f32(w[k], p.act, p.alpha);
          if (p.dact) {
            const i32x4 tz = *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[2 * e] *= act_dz(__uint_as_float(((uint32_t)tz[e]) << 16), p.dact, p.alpha);
              w[2 * e + 1] *= act_dz(__uint_as_float(((uint32_t)tz[e]) & 0xffff0000u), p.dact, p.alpha);
            }
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
          narrow_act(w, p.act, p.alpha);
          if (p.dact) {
            const i32x4 tz = *(const i32x4*)((const bf16_t*)p.z + pix * p.z_ld + co);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[2 * e] *= act_dz(__uint_as_float(((uint32_t)tz[e]) << 16), p.dact, p.alpha);
              w[2 * e + 1] *= act_dz(__uint_as_float(((uint32_t)tz[e]) & 0xffff0000u), p.dact, p.alpha);
            }
          }
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (int)pk2_bf16(w[2 * e], w[2 * e + 1]);
          *(i32x4*)dst = o;
        }
      }
    }
  }
}

// DVIE_CONV_NARROW=0: these layers on the chunked halo kernel (A/B runs); read per launch
static bool narrow_env_on() {
  const char* e = getenv("DVIE_CONV_NARROW");
  return !(e && *e == '0');
}

// DVIE_NARROW_DBG (timing only, wrong results; -DDVIE_TIMING_DBG builds only): bit 1 = no operand DMA, bit 2 = no MFMAs
static int narrow_dbg() {
#ifdef DVIE_TIMING_DBG
  const char* e = getenv("DVIE_NARROW_DBG");
  return e && *e ? atoi(e) : 0;
#else
  return 0;
#endif
}

// Returns true when the narrow-output kernel took the launch.
bool conv_narrow_launch(const dvie_conv_desc& p, hipStream_t s) {
  if (p.dtype != DVIE_BF16 || !narrow_env_on()) return false;
  if (p.th != 3 || p.tw != 3 || p.sy != 1 || p.sx != 1 || p.ddy != 1 || p.ddx != 1) return false;
  if (p.cout > 32 || p.cout % 8 != 0 || p.c <= 64 || p.c % 32 != 0 || p.kpad < 9 * p.c) return false;
  if (p.osy != 1 || p.osx != 1 || p.ory != 0 || p.orx != 0 || p.yh != p.oh || p.yw != p.ow) return false;
  const unsigned long long npx = (unsigned long long)p.n * p.ih * p.iw;
  if (npx >= (1ull << 31) || ((npx - 1) * (unsigned long long)p.x_ld + p.c) * 2ull >= 0xFFFFFF00ull) return false;
  if ((unsigned long long)p.cout * p.kpad * 2ull >= 0xFFFFFF00ull) return false;
  typedef NarrowCfg C;
  const int tiles_x = (p.ow + C::TW - 1) / C::TW, tiles_y = (p.oh + C::NW - 1) / C::NW;
  const long long nt = (long long)tiles_x * tiles_y * p.n;
  if (nt >= (1LL << 30)) return false;
  const int n_tiles = (int)nt;
  const int grid = n_tiles < 256 ? n_tiles : 256;  // one 150-KB workgroup per CU
  if (p.out_f32)
    DVIE_LAUNCH(conv_narrow_kernel<true>, dim3(grid), dim3(512), 0, s, p, tiles_x, tiles_y, n_tiles, narrow_dbg());
  else
    DVIE_LAUNCH(conv_narrow_kernel<false>, dim3(grid), dim3(512), 0, s, p, tiles_x, tiles_y, n_tiles, narrow_dbg());
  return true;
}

}  // namespace dvie
