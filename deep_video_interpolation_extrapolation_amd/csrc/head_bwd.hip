// Fused backward of the narrow-output 3x3 head convs for gfx950, bf16: HRNet's
// rgb_layer[2] / seg_layer[2] (448 -> 3 / 448 -> 20, reference nets/HRNet.py:410-442 and
// 584-588) together with the LeakyReLU derivative of the hidden map they read.
//
// Per layer the unfused backward reads the 448-channel hidden map h twice (a data-gradient
// conv whose epilogue applies LeakyReLU'(h), and a weight-gradient kernel) and streams the
// tiny output gradient g.  Here one kernel reads h once:
//   D[p][(t, o)] = g[p + (dy0 + i_t, dx0 + j_t)][o]        (t = 3 i_t + j_t, zero outside)
//   dh[p][ci]    = act'(h[p][ci]) * sum_k D[p][k] * wd[ci][k]           (GEMM 1, K = 9 cout)
//   part[s][o][(8 - t) c + ci] += sum_{p in split s} D[p][(t, o)] h[p][ci]  (GEMM 2, K = pixels)
// A workgroup (8 waves) owns one 64-channel block of h and a contiguous range of 4-row x
// 64-pixel tiles.  Per tile it stages by LDS-DMA (double buffered, the next tile streams in
// while this one computes) the h tile [256 px][64 ch] (128-B rows, 16-B chunks XOR-swizzled
// by bit 1 of the pixel so the transposed reads are conflict-free) and the output-gradient
// halo [6 x 66 px][cout] (zeros outside the image: the conv padding).  D is never formed:
// GEMM 1 reads its B fragments (8 consecutive k = 8 channels of one tap) straight from the
// halo at the tap's shift, GEMM 2 its A fragments (8 consecutive pixels of one k) with
// ds_read_b64_tr_b16 transposed reads of the same image; GEMM 2's B fragments are transposed
// reads of the h tile, which also supplies act'(h) for GEMM 1's epilogue.  The data-gradient
// weights of the block stay in LDS for the whole launch.  GEMM 2's accumulators live in
// registers across the tiles and are written once as this split's partial slab (the
// dvie_conv2d_wgrad layout, reduced by dvie_wgrad_reduce).
//
// MFMA v_mfma_f32_32x32x16_bf16.  GEMM 1: wave (row wr, channel half wc) computes
// dh^T[32 ch][64 px] (A = weights, B = halo).  GEMM 2: wave (ci block nb, k-row blocks mq and
// mq + 4) over all 256 pixels of the tile.
#include <algorithm>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 hb_bf16x2 __attribute__((ext_vector_type(2)));
typedef float hb_f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_hb;

template <int CO>
struct HbCfg {
  static constexpr int NW = 8, R = 4, TW = 64;
  static constexpr int KC = 9 * CO / 8;                  // 16-B chunks of one pixel's D row
  static constexpr int KS = (KC + 1) / 2;                 // 16-wide k slices of GEMM 1
  static constexpr int NMB = (9 * CO + 31) / 32;          // 32-row k blocks of GEMM 2
  static constexpr int WPITCH = KS * 32 + 16;             // weight LDS row pitch (bytes)
  static constexpr int WSZ = 64 * WPITCH;
  static constexpr int HT = R * TW * 128;                 // h tile: 256 px x 128 B
  static constexpr int HPC = HT / 1024;                   // its 1-KB DMA pieces
  static constexpr int HR = R + 2, HWD = TW + 2;          // output-gradient halo rows / columns
  static constexpr int GREC = CO * 2;                     // halo bytes per pixel
  static constexpr int GPC = (HR * HWD * GREC / 16 + 63) / 64;
  static constexpr int GQ = (GPC + NW - 1) / NW;          // halo pieces per wave (upper bound)
  static constexpr int STAGE = HT + GPC * 1024;
  // stage buffers: three for cout 8 (tile t + 2 streams in while tile t computes: one tile of
  // compute did not cover a tile's DMA latency + transfer), two for cout 24 (three do not fit)
  static constexpr int NSTG = WSZ + 3 * STAGE <= 163840 ? 3 : 2;
  static constexpr int SMEM = WSZ + NSTG * STAGE;
  // DMA pieces a wave issues per tile (h tile + its share of the halo)
  __host__ __device__ static constexpr int pieces(int wave) { return HPC / NW + (wave < GPC % NW || GPC % NW == 0 ? GQ : GQ - 1); }
  // GEMM 1 B-fragment offset of k-chunk kc inside the halo (tap shift + channel chunk); the
  // zero-weight padding chunk of cout 8 reads tap 8 (finite data times zero weights)
  __host__ __device__ static constexpr int chunk_off(int kc) {
    const int k = kc < KC ? kc : KC - 1;
    const int t = k / (CO / 8), oc = k % (CO / 8);
    return ((t / 3) * HWD + t % 3) * GREC + oc * 16;
  }
};

__device__ __forceinline__ bf16x8 hb_tr_pair(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ uint32_t hb_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hb_f32x2{a, b}), hb_bf16x2));
}

// s_waitcnt vmcnt(n) for a wave-uniform n < 32 (the DMA is inline asm: the compiler counts
// none of it, so the kernel waits for its own pieces explicitly)
#define DVIE_HB_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4) | (15 << 8))
__device__ __forceinline__ void hb_wait_vmcnt(int n) {
  switch (n) {
#define DVIE_HB_CASE(N) \
  case N:               \
    DVIE_HB_VMCNT(N);   \
    break;
    DVIE_HB_CASE(1) DVIE_HB_CASE(2) DVIE_HB_CASE(3) DVIE_HB_CASE(4) DVIE_HB_CASE(5) DVIE_HB_CASE(6) DVIE_HB_CASE(7)
    DVIE_HB_CASE(8) DVIE_HB_CASE(9) DVIE_HB_CASE(10) DVIE_HB_CASE(11) DVIE_HB_CASE(12) DVIE_HB_CASE(13) DVIE_HB_CASE(14)
    DVIE_HB_CASE(15) DVIE_HB_CASE(16) DVIE_HB_CASE(17) DVIE_HB_CASE(18) DVIE_HB_CASE(19) DVIE_HB_CASE(20)
#undef DVIE_HB_CASE
    default: __builtin_amdgcn_s_waitcnt(0);
  }
}

template <int CO>
__global__ __launch_bounds__(512) void head3_bwd_kernel(const dvie_head3_bwd_desc p, int n_cb, int tiles_x,
                                                        int tiles_y, int n_tiles) {
  typedef HbCfg<CO> C;
  constexpr int NW = C::NW;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // workgroup -> (channel block, split); the blocks of one split are XCD-neighbours
  // (blocks b and b + 8 share an XCD under round-robin dispatch), so they share g in L2
  const int G = gridDim.x, xg = blockIdx.x & 7, xi = blockIdx.x >> 3;
  const int q8 = G >> 3, r8 = G & 7;
  const int lid = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + xi;
  const int cb = lid % n_cb, split = lid / n_cb;
  const int t_begin = (int)((long long)split * n_tiles / p.splits);
  const int t_end = (int)((long long)(split + 1) * n_tiles / p.splits);

  char* const Wl = smem;
  char* const St = smem + C::WSZ;

  // ---- this block's data-gradient weights [64 ci][KS * 16 k] into LDS, once ----
  for (int i = tid; i < 64 * C::KS * 2; i += NW * 64) {
    const int r = i / (C::KS * 2), ch = i - r * (C::KS * 2);
    const i32x4 v = *(const i32x4*)((const bf16_t*)p.wd + (size_t)(cb * 64 + r) * p.kpad + ch * 8);
    *(i32x4*)(Wl + r * C::WPITCH + ch * 16) = v;
  }

  // ---- per-lane DMA geometry (tile independent) ----
  int hgeo[C::HPC / NW];
#pragma unroll
  for (int q = 0; q < C::HPC / NW; ++q) {
    const int slot = (wave + NW * q) * 64 + lane, P = slot >> 3;
    hgeo[q] = (P << 4) | ((slot & 7) ^ (4 * ((P >> 1) & 1)));
  }
  int ggeo[C::GQ];
#pragma unroll
  for (int q = 0; q < C::GQ; ++q) {
    const int slot = (wave + NW * q) * 64 + lane, px = slot / (CO / 8), ch = slot % (CO / 8);
    ggeo[q] = px < C::HR * C::HWD ? ((px / C::HWD) << 16) | ((px % C::HWD) << 4) | ch : -1;
  }
  const unsigned hrow = (unsigned)p.h_ld * 2u, grow = (unsigned)p.g_ld * 2u;
  const unsigned long long npx = (unsigned long long)p.n * p.hgt * p.wid;
  const unsigned hbytes = (unsigned)((npx - 1) * p.h_ld * 2ull + (unsigned long long)p.c * 2ull - cb * 128ull);
  const unsigned gbytes = (unsigned)((npx - 1) * p.g_ld * 2ull + (unsigned long long)CO * 2ull);
  const __amdgpu_buffer_rsrc_t rh =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.h + cb * 128), 0, (int)hbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, 0, (int)gbytes, 0x00020000);

  struct Tile {
    int n, y0, x0;
  };
  auto tile_of = [&](int t) {
    Tile T;
    T.x0 = (t % tiles_x) * C::TW;
    t /= tiles_x;
    T.y0 = (t % tiles_y) * C::R;
    T.n = t / tiles_y;
    return T;
  };
  auto issue = [&](int t, int sb) {
    const Tile T = tile_of(t);
    char* S = St + sb * C::STAGE;
#pragma unroll
    for (int q = 0; q < C::HPC / NW; ++q) {
      const int gq = hgeo[q], P = gq >> 4;
      const int y = T.y0 + (P >> 6), x = T.x0 + (P & 63);
      const bool ok = y < p.hgt && x < p.wid;
      const unsigned o = ok ? (unsigned)((T.n * p.hgt + y) * p.wid + x) * hrow + (unsigned)(gq & 15) * 16u : OOB;
      lds_dma16(rh, S + (wave + NW * q) * 1024, o);
    }
#pragma unroll
    for (int q = 0; q < C::GQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::GPC) continue;  // (wave-uniform)
      const int v = ggeo[q];
      const int iy = T.y0 + p.dy0 + ((v >> 16) & 0xFF), ix = T.x0 + p.dx0 + ((v >> 4) & 0xFFF);
      const bool ok = v >= 0 && (unsigned)iy < (unsigned)p.hgt && (unsigned)ix < (unsigned)p.wid;
      const unsigned o = ok ? (unsigned)((T.n * p.hgt + iy) * p.wid + ix) * grow + (unsigned)(v & 15) * 16u : OOB;
      lds_dma16(rg, S + C::HT + pc * 1024, o);
    }
  };

  // ---- fragment geometry ----
  // GEMM 1: wave (row wr, channel half wc); A = weight rows 32 wc + r32, B = halo pixel
  // (wr + i_t, 32 b + r32 + j_t) of k-chunk 2 s + hh
  const int wr = wave & 3, wc = wave >> 2;
  const int a1_base = (32 * wc + r32) * C::WPITCH + hh * 16;
  const int b1_base = (wr * C::HWD + r32) * C::GREC;
  // GEMM 2: wave (ci block nb, k-row blocks mb0 = mq, mb1 = mq + 4); transposed reads: lane
  // 4 q + pq of 16-lane group g4 addresses pixel row q of the group's 4-pixel block and
  // columns 4 pq .. 4 pq + 3 (k for A, ci for B) of its 16-column block
  const int nb = wave & 1, mq = wave >> 1;
  const bool has0 = mq < C::NMB, has1 = mq + 4 < C::NMB;
  const int g4 = lane >> 4, li = lane & 15, qq = li >> 2, pq = li & 3;
  const int pix_l = 8 * (g4 >> 1) + qq;  // lane's pixel within a 16-pixel slice (+ 4 r)
  auto k_off = [&](int mb) {  // halo offset of the lane's 4 k values (tap shift + channel)
    const int m0 = 32 * mb + 16 * (g4 & 1) + 4 * pq;
    int t = m0 / CO;
    const int o0 = m0 - t * CO;
    t = t < 9 ? t : 8;  // k rows past 9 cout: finite data, results discarded
    return ((t / 3) * C::HWD + t % 3) * C::GREC + o0 * 2;
  };
  const int a2_off0 = pix_l * C::GREC + k_off(has0 ? mq : 0);
  const int a2_off1 = pix_l * C::GREC + k_off(has1 ? mq + 4 : 0);
  const int ci0 = 32 * nb + 16 * (g4 & 1) + 4 * pq;
  const int b2_off = pix_l * 128 + (((ci0 >> 3) ^ (4 * ((qq >> 1) & 1))) << 4) + (ci0 & 7) * 2;

  f32x16 acc2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc2[j][e] = 0.f;

  // output-gradient stores: buffer stores every wave issues (out-of-image pixels at an
  // out-of-range offset, dropped), so the vector-memory count of a tile is fixed
  const __amdgpu_buffer_rsrc_t rdh =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dh, 0, (int)(npx * p.dh_ld * 2ull), 0x00020000);
  constexpr int NSTG = C::NSTG, NST = 4;  // stage buffers; dh stores per wave per tile
  const int np = C::pieces(wave);
  const int ntl = t_end - t_begin;
#pragma unroll
  for (int j = 0; j < NSTG - 1; ++j)
    if (j < ntl) issue(t_begin + j, j);
  for (int t = t_begin; t < t_end; ++t) {
    const int li = t - t_begin;
    const int sb = li % NSTG;
    // this tile's DMA (and the weight stores) have landed for every wave, and every wave is
    // done reading the buffer tile t + NSTG - 1 streams into.  Issued after this tile's
    // pieces (in order): tiles li + 1 .. li + NSTG - 2 and the stores of tiles li - NSTG + 1 ..
    // li - 1 (interleaved), which may stay in flight.
    if (NSTG == 2) {
      __builtin_amdgcn_s_waitcnt(0);
    } else {
      const int later = (li + 1 < ntl ? np : 0) + (li >= 1 ? NST : 0) + (li >= 2 ? NST : 0);
      if (later == 0)
        __builtin_amdgcn_s_waitcnt(0);
      else
        hb_wait_vmcnt(later);
    }
    __builtin_amdgcn_s_barrier();
    if (t + NSTG - 1 < t_end) issue(t + NSTG - 1, (li + NSTG - 1) % NSTG);
    const char* S = St + sb * C::STAGE;
    const char* Gh = S + C::HT;
    const Tile T = tile_of(t);

    // ---- GEMM 1: dh^T[32 ch][64 px] of this wave ----
    f32x16 acc1[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc1[b][e] = 0.f;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      const i32x4 a = *(const i32x4*)(Wl + a1_base + s * 32);
      const int boff = hh ? C::chunk_off(2 * s + 1) : C::chunk_off(2 * s);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const i32x4 bv = *(const i32x4*)(Gh + b1_base + 32 * b * C::GREC + boff);
        acc1[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, bv),
                                                          acc1[b], 0, 0, 0);
      }
    }

    // ---- GEMM 2: partial dW over the tile's 256 pixels ----
    // (slice sl + 1's fragments are read while slice sl's MFMAs run)
    {
      bf16x8 fb[2], fa0[2], fa1[2];
      auto ld2 = [&](int sl, int buf) {
        const int pa = ((sl >> 2) * C::HWD + 16 * (sl & 3)) * C::GREC;  // slice's first pixel in the halo
        fb[buf] = hb_tr_pair(S + b2_off + 16 * sl * 128, S + b2_off + (16 * sl + 4) * 128);
        if (has0) fa0[buf] = hb_tr_pair(Gh + a2_off0 + pa, Gh + a2_off0 + pa + 4 * C::GREC);
        if (has1) fa1[buf] = hb_tr_pair(Gh + a2_off1 + pa, Gh + a2_off1 + pa + 4 * C::GREC);
      };
      ld2(0, 0);
#pragma unroll
      for (int sl = 0; sl < 16; ++sl) {
        if (sl + 1 < 16) ld2(sl + 1, (sl + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        if (has0) acc2[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0[sl & 1], fb[sl & 1], acc2[0], 0, 0, 0);
        if (has1) acc2[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1[sl & 1], fb[sl & 1], acc2[1], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // ---- GEMM 1 epilogue: permlane32 pairing -> 8 consecutive channels of one pixel per
    // lane; times act'(h) (h from the staged tile); bf16 store ----
    const int oy = T.y0 + wr;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float v[2][8];
#pragma unroll
      for (int P = 0; P < 2; ++P)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc1[b][8 * P + e]),
                                                           __float_as_uint(acc1[b][8 * P + 4 + e]), false, false);
          v[P][e] = __uint_as_float(sw[0]);
          v[P][4 + e] = __uint_as_float(sw[1]);
        }
      const int px = wr * 64 + 32 * b + r32;  // pixel within the tile
      const int ox = T.x0 + 32 * b + r32;
      const bool in = oy < p.hgt && ox < p.wid;
      const long long pix = ((long long)T.n * p.hgt + oy) * p.wid + ox;
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const int c8 = 4 * wc + 2 * P + hh;
        float* w = v[P];
        if (p.dact) {
          const i32x4 hz = *(const i32x4*)(S + px * 128 + ((c8 ^ (4 * ((px >> 1) & 1))) << 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            w[2 * e] *= act_dz(__uint_as_float(((uint32_t)hz[e]) << 16), p.dact, p.alpha);
            w[2 * e + 1] *= act_dz(__uint_as_float(((uint32_t)hz[e]) & 0xffff0000u), p.dact, p.alpha);
          }
        }
        i32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (int)hb_pack(w[2 * e], w[2 * e + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(
            o, rdh, in ? (unsigned)((pix * p.dh_ld + cb * 64 + 8 * c8) * 2) : OOB, 0, 0);
      }
    }
  }

  // ---- this split's partial slab: part[split][o][(8 - t) c + ci], rows k = 9 cout only ----
  const long long kstride = 9ll * p.c;
  float* slab = p.ws + (long long)split * CO * kstride + cb * 64 + 32 * nb + r32;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (!(j == 0 ? has0 : has1)) continue;
    const int mb = j == 0 ? mq : mq + 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 32 * mb + 8 * i + 4 * hh + e;
        const int tt = k / CO, o = k - tt * CO;
        if (tt < 9) slab[o * kstride + (8 - tt) * p.c] = acc2[j][4 * i + e];
      }
  }
}

}  // namespace dvie

extern "C" int dvie_head3_bwd(const dvie_head3_bwd_desc* d, void* stream) {
  using namespace dvie;
  DVIE_CHECK_ARG(d && d->g && d->h && d->wd && d->dh && d->ws, "head3_bwd: null pointer");
  DVIE_CHECK_ARG(d->cout == 8 || d->cout == 24, "head3_bwd: cout %d (8 or 24)", d->cout);
  DVIE_CHECK_ARG(d->c > 0 && d->c % 64 == 0 && d->n > 0 && d->hgt > 0 && d->wid > 0, "head3_bwd: shape");
  DVIE_CHECK_ARG(d->dact == DVIE_ACT_NONE || d->dact == DVIE_ACT_LRELU, "head3_bwd: dact %d", d->dact);
  DVIE_CHECK_ARG(d->splits > 0 && d->g_ld >= d->cout && d->h_ld >= d->c && d->dh_ld >= d->c, "head3_bwd: args");
  const int ks16 = (d->cout == 8 ? HbCfg<8>::KS : HbCfg<24>::KS) * 16;
  DVIE_CHECK_ARG(d->kpad >= ks16 && d->kpad % 8 == 0, "head3_bwd: kpad %d < %d", d->kpad, ks16);
  const unsigned long long npx = (unsigned long long)d->n * d->hgt * d->wid;
  DVIE_CHECK_ARG(npx * (unsigned long long)std::max(std::max(d->h_ld, d->g_ld), d->dh_ld) * 2ull < 0xFFFFFF00ull,
                 "head3_bwd: maps exceed the 32-bit buffer range");
  const int tiles_x = (d->wid + 63) / 64, tiles_y = (d->hgt + 3) / 4;
  const long long nt = (long long)tiles_x * tiles_y * d->n;
  DVIE_CHECK_ARG(nt < (1LL << 30), "head3_bwd: too many tiles");
  const int n_cb = d->c / 64;
  const int grid = n_cb * d->splits;
  hipStream_t s = (hipStream_t)stream;
  if (d->cout == 8)
    DVIE_LAUNCH(head3_bwd_kernel<8>, dim3(grid), dim3(512), 0, s, *d, n_cb, tiles_x, tiles_y, (int)nt);
  else
    DVIE_LAUNCH(head3_bwd_kernel<24>, dim3(grid), dim3(512), 0, s, *d, n_cb, tiles_x, tiles_y, (int)nt);
  DVIE_RETURN_LAUNCH();
}
