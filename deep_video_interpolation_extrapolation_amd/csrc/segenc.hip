// Fused forward of HRNet's segmentation encoder for gfx950, bf16 (reference nets/HRNet.py:
// 358-364 seg_encoder = conv3x3(20 -> 32) + ELU, conv3x3(32 -> 32) + ELU, conv3x3(32 -> 4),
// run on each input segmentation map at l.533-537):
//   e1 = ELU(conv0(seg) + b0),  e2 = ELU(conv2(e1) + b2),  out = conv4(e2) + b4
// Unfused, three launches stream the 24-channel input and the two 32-channel intermediates
// through HBM between tiny convs (K = 216 / 288, N = 32 / 8) that cannot fill the chip.  Here
// a workgroup owns a 4-row x 64-pixel output tile: it stages the input halo (10 x 70 px) once,
// computes e1 on the 8 x 68 region the next conv needs and e2 on 6 x 66, both kept in LDS
// (zero outside the image: the next conv's padding), and the output on the tile.  e1 and e2
// are still written once (the backward reads them), the input is read once, and the 4-channel
// result goes straight into its slice of the stem buffer.  Recompute: e1 2.1x, e2 1.55x of
// the tile (a few tens of kFLOP per pixel; the launch was bound by its traffic and latency).
//
// MFMA v_mfma_f32_32x32x16_bf16 per 32-pixel block of a stage's region (flattened row-major,
// so blocks span rows): A = weights (32 output channels x 16 k; conv4's 8 real rows, the
// others read a clamped row and are discarded), B = the source image at the tap's shift
// (8 consecutive channels of one pixel per lane).  Epilogue: permlane32 pairing gives a lane 8
// consecutive channels of one pixel, + bias, ELU, bf16.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 se_bf16x2 __attribute__((ext_vector_type(2)));
typedef float se_f32x2 __attribute__((ext_vector_type(2)));

namespace dvie {

typedef __attribute__((address_space(3))) void* lds_ptr_se;

struct SeCfg {
  static constexpr int NW = 8, R = 4, TW = 64;
  // regions: input (R+6) x (TW+6), e1 (R+4) x (TW+4), e2 (R+2) x (TW+2), out R x TW
  static constexpr int IN_W = TW + 6, IN_H = R + 6, IN_PITCH = 48;   // 24 bf16 channels
  static constexpr int E1_W = TW + 4, E1_H = R + 4, E_PITCH = 80;    // 32 channels + 16-B pad
  static constexpr int E2_W = TW + 2, E2_H = R + 2;
  static constexpr int IN_SZ = IN_H * IN_W * IN_PITCH;
  static constexpr int IN_PC = (IN_SZ / 16 + 63) / 64;                // 1-KB DMA pieces
  static constexpr int E1_SZ = E1_H * E1_W * E_PITCH;
  static constexpr int E2_SZ = E2_H * E2_W * E_PITCH;
  // weights [co][k] with a 16-B pad per row: conv0 K = 9*24 = 216 (14 slices), conv2 / conv4
  // K = 9*32 = 288 (18 slices)
  static constexpr int KS0 = 14, KS2 = 18;
  static constexpr int W0_PITCH = KS0 * 32 + 16, W2_PITCH = KS2 * 32 + 16;
  static constexpr int W0_SZ = 32 * W0_PITCH, W2_SZ = 32 * W2_PITCH, W4_SZ = 8 * W2_PITCH;
  static constexpr int O_W0 = 0, O_W2 = W0_SZ, O_W4 = O_W2 + W2_SZ, O_IN = O_W4 + W4_SZ;
  static constexpr int O_E1 = O_IN + IN_PC * 1024, O_E2 = O_E1 + E1_SZ;
  static constexpr int SMEM = O_E2 + E2_SZ;
};
static_assert(SeCfg::SMEM <= 163840, "segenc LDS");

__device__ __forceinline__ uint32_t se_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((se_f32x2{a, b}), se_bf16x2));
}

// One conv stage over a flattened region of `npx` pixels of width RW: output pixel q = (r, c)
// reads the source region (width RW + 2, pitch SP, CPT 16-B chunks per pixel) at (r + i, c + j).
// Each wave takes 32-pixel blocks round-robin, two at a time (blocks blk and blk + NW: the
// weight fragment of a k-step serves both and their MFMA chains interleave); `epi(q,
// lane_channels, v[8])` consumes the 8 consecutive channels 16 P + 8 hh .. +7 (P = 0, 1) of
// pixel q.
template <int KS, int CPT, int RW, int SP, int WP, typename Epi>
__device__ __forceinline__ void se_stage(const char* Wl, int wrows, const char* Src, int npx, int wave, int lane,
                                         Epi&& epi) {
  constexpr int SW = RW + 2;
  constexpr int KC = 9 * CPT;
  const int r32 = lane & 31, hh = lane >> 5;
  const char* Wa = Wl + (r32 < wrows ? r32 : r32 & (wrows - 1)) * WP + hh * 16;
  const int nblk = (npx + 31) / 32;
  auto run = [&](int blk0, auto nbt) {
    constexpr int NB = decltype(nbt)::value;
    int q[NB];
    const char* B[NB];
    f32x16 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      q[b] = (blk0 + SeCfg::NW * b) * 32 + r32;
      const int qc = q[b] < npx ? q[b] : npx - 1;  // (pad lanes read a valid pixel, results dropped)
      const int r = qc / RW, c = qc - r * RW;
      B[b] = Src + (r * SW + c) * SP;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    }
    // (k-step s + 1's fragments are read while step s's MFMAs run)
    i32x4 fa[2], fb[2][NB];
    auto ld = [&](int s, int buf) {
      fa[buf] = *(const i32x4*)(Wa + s * 32);
      int kc = 2 * s + hh;
      kc = kc < KC ? kc : KC - 1;  // zero-weight padding chunk: any finite source
      const int t = kc / CPT, cc = kc - t * CPT;
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[buf][b] = *(const i32x4*)(B[b] + ((t / 3) * SW + t % 3) * SP + cc * 16);
    };
    ld(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) ld(s + 1, (s + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[s & 1]),
                                                         __builtin_bit_cast(bf16x8, fb[s & 1][b]), acc[b], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
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
      if (q[b] < npx) epi(q[b] / RW, q[b] % RW, v);
    }
  };
  for (int blk = wave; blk < nblk; blk += 2 * SeCfg::NW) {
    if (blk + SeCfg::NW < nblk)
      run(blk, std::integral_constant<int, 2>());
    else
      run(blk, std::integral_constant<int, 1>());
  }
}

__global__ __launch_bounds__(512) void segenc_fwd_kernel(const dvie_segenc_desc p, int tiles_x, int tiles_y,
                                                         int n_tiles) {
  typedef SeCfg C;
  constexpr int NW = C::NW;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // ---- weights into LDS, once: conv0 [32][216 -> 224], conv2 [32][288], conv4 [8][288] ----
  auto wload = [&](const bf16_t* w, int kpad, int rows, int chunks, int pitch, int off) {
    for (int i = tid; i < rows * chunks; i += NW * 64) {
      const int r = i / chunks, ch = i - r * chunks;
      *(i32x4*)(smem + off + r * pitch + ch * 16) = *(const i32x4*)(w + (size_t)r * kpad + ch * 8);
    }
  };
  wload((const bf16_t*)p.w0, p.kpad0, 32, 2 * C::KS0, C::W0_PITCH, C::O_W0);
  wload((const bf16_t*)p.w2, p.kpad2, 32, 2 * C::KS2, C::W2_PITCH, C::O_W2);
  wload((const bf16_t*)p.w4, p.kpad4, 8, 2 * C::KS2, C::W2_PITCH, C::O_W4);

  // input DMA geometry: slot -> (halo row, column, 16-B chunk of the 48-B pixel)
  constexpr int IQ = (C::IN_PC + NW - 1) / NW;
  int igeo[IQ];
#pragma unroll
  for (int q = 0; q < IQ; ++q) {
    const int slot = (wave + NW * q) * 64 + lane, px = slot / 3, ch = slot - 3 * px;
    igeo[q] = px < C::IN_H * C::IN_W ? ((px / C::IN_W) << 16) | ((px % C::IN_W) << 4) | ch : -1;
  }
  const unsigned long long npx = (unsigned long long)p.n * p.h * p.w;
  const unsigned irow = (unsigned)p.in_ld * 2u;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.in, 0, (int)((npx - 1) * p.in_ld * 2ull + 48ull), 0x00020000);

  // biases in registers (a lane's epilogue channels: 16 P + 8 hh .. +7)
  float bb0[2][8], bb2[2][8], bb4[8];
#pragma unroll
  for (int P = 0; P < 2; ++P)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bb0[P][e] = p.b0[16 * P + 8 * hh + e];
      bb2[P][e] = p.b2[16 * P + 8 * hh + e];
    }
#pragma unroll
  for (int e = 0; e < 8; ++e) bb4[e] = p.b4[e];

  // The next tile's input halo is loaded into registers while this tile's three stages run
  // and written to LDS at the next tile's start (its global latency hides behind the MFMAs).
  i32x4 stg[IQ];
  auto tile_pos = [&](int t, int& n, int& y0, int& x0) {
    int tt = t;
    x0 = (tt % tiles_x) * C::TW;
    tt /= tiles_x;
    y0 = (tt % tiles_y) * C::R;
    n = tt / tiles_y;
  };
  auto load_tile = [&](int t) {
    int n, y0, x0;
    tile_pos(t, n, y0, x0);
#pragma unroll
    for (int q = 0; q < IQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::IN_PC) continue;  // (wave-uniform)
      const int v = igeo[q];
      const int iy = y0 - 3 + ((v >> 16) & 0xFF), ix = x0 - 3 + ((v >> 4) & 0xFFF);
      const bool ok = v >= 0 && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
      const unsigned o = ok ? (unsigned)((n * p.h + iy) * p.w + ix) * irow + (unsigned)(v & 15) * 16u : OOB;
      stg[q] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rin, o, 0, 0));
    }
  };
  const int G = gridDim.x;
  if ((int)blockIdx.x < n_tiles) load_tile(blockIdx.x);
  for (int t = blockIdx.x; t < n_tiles; t += G) {
    int n, y0, x0;
    tile_pos(t, n, y0, x0);
    // previous tile's readers are done with every image (and the weights have landed)
    __syncthreads();
#pragma unroll
    for (int q = 0; q < IQ; ++q) {
      const int pc = wave + NW * q;
      if (pc < C::IN_PC) *(i32x4*)(smem + C::O_IN + pc * 1024 + lane * 16) = stg[q];
    }
    __syncthreads();
    if (t + G < n_tiles) load_tile(t + G);

    // ---- e1 on the 8 x 68 region at (y0 - 2, x0 - 2) ----
    se_stage<C::KS0, 3, C::E1_W, C::IN_PITCH, C::W0_PITCH>(
        smem + C::O_W0, 32, smem + C::O_IN, C::E1_H * C::E1_W, wave, lane, [&](int r, int c, float (*v)[8]) {
          const int gy = y0 - 2 + r, gx = x0 - 2 + c;
          const bool in = (unsigned)gy < (unsigned)p.h && (unsigned)gx < (unsigned)p.w;
          const bool interior = r >= 2 && r < 2 + C::R && c >= 2 && c < 2 + C::TW && in;
#pragma unroll
          for (int P = 0; P < 2; ++P) {
            const int co = 16 * P + 8 * hh;
            i32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = in ? elu_bf(v[P][2 * e] + bb0[P][2 * e]) : 0.f;
              const float b = in ? elu_bf(v[P][2 * e + 1] + bb0[P][2 * e + 1]) : 0.f;
              o[e] = (int)se_pack(a, b);
            }
            *(i32x4*)(smem + C::O_E1 + (r * C::E1_W + c) * C::E_PITCH + co * 2) = o;
            if (interior) *(i32x4*)((bf16_t*)p.e1 + ((long long)(n * p.h + gy) * p.w + gx) * p.e1_ld + co) = o;
          }
        });
    __syncthreads();
    // ---- e2 on the 6 x 66 region at (y0 - 1, x0 - 1) ----
    se_stage<C::KS2, 4, C::E2_W, C::E_PITCH, C::W2_PITCH>(
        smem + C::O_W2, 32, smem + C::O_E1, C::E2_H * C::E2_W, wave, lane, [&](int r, int c, float (*v)[8]) {
          const int gy = y0 - 1 + r, gx = x0 - 1 + c;
          const bool in = (unsigned)gy < (unsigned)p.h && (unsigned)gx < (unsigned)p.w;
          const bool interior = r >= 1 && r < 1 + C::R && c >= 1 && c < 1 + C::TW && in;
#pragma unroll
          for (int P = 0; P < 2; ++P) {
            const int co = 16 * P + 8 * hh;
            i32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = in ? elu_bf(v[P][2 * e] + bb2[P][2 * e]) : 0.f;
              const float b = in ? elu_bf(v[P][2 * e + 1] + bb2[P][2 * e + 1]) : 0.f;
              o[e] = (int)se_pack(a, b);
            }
            *(i32x4*)(smem + C::O_E2 + (r * C::E2_W + c) * C::E_PITCH + co * 2) = o;
            if (interior) *(i32x4*)((bf16_t*)p.e2 + ((long long)(n * p.h + gy) * p.w + gx) * p.e2_ld + co) = o;
          }
        });
    __syncthreads();
    // ---- out (8 channels: 4 real, 4 zero-weight) on the tile ----
    se_stage<C::KS2, 4, C::TW, C::E_PITCH, C::W2_PITCH>(
        smem + C::O_W4, 8, smem + C::O_E2, C::R * C::TW, wave, lane, [&](int r, int c, float (*v)[8]) {
          const int gy = y0 + r, gx = x0 + c;
          if (hh || gy >= p.h || gx >= p.w) return;  // channels 0..7 = pair 0, lane half 0
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (int)se_pack(v[0][2 * e] + bb4[2 * e], v[0][2 * e + 1] + bb4[2 * e + 1]);
          *(i32x4*)((bf16_t*)p.out + ((long long)(n * p.h + gy) * p.w + gx) * p.out_ld) = o;
        });
  }
}

}  // namespace dvie

extern "C" int dvie_segenc_fwd(const dvie_segenc_desc* d, void* stream) {
  using namespace dvie;
  DVIE_CHECK_ARG(d && d->in && d->e1 && d->e2 && d->out && d->w0 && d->w2 && d->w4, "segenc: null pointer");
  DVIE_CHECK_ARG(d->b0 && d->b2 && d->b4, "segenc: biases required");
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0, "segenc: shape");
  DVIE_CHECK_ARG(d->in_ld >= 24 && d->e1_ld >= 32 && d->e2_ld >= 32 && d->out_ld >= 8, "segenc: leading dims");
  DVIE_CHECK_ARG(d->kpad0 >= 224 && d->kpad2 >= 288 && d->kpad4 >= 288, "segenc: kpad");
  const unsigned long long npx = (unsigned long long)d->n * d->h * d->w;
  DVIE_CHECK_ARG(npx * (unsigned long long)d->in_ld * 2ull < 0xFFFFFF00ull && npx < (1ull << 31),
                 "segenc: input exceeds the 32-bit buffer range");
  const int tiles_x = (d->w + 63) / 64, tiles_y = (d->h + 3) / 4;
  const long long nt = (long long)tiles_x * tiles_y * d->n;
  DVIE_CHECK_ARG(nt < (1LL << 30), "segenc: too many tiles");
  const int grid = (int)(nt < 256 ? nt : 256);  // one 147-KB workgroup per CU, tiles round-robin
  DVIE_LAUNCH(segenc_fwd_kernel, dim3(grid), dim3(512), 0, (hipStream_t)stream, *d, tiles_x, tiles_y, (int)nt);
  DVIE_RETURN_LAUNCH();
}

// ============================================================================================
// Fused backward of the segmentation encoder (the three convs above; the encoder input needs
// no gradient).  Per 4 x 64 tile, with dout = the gradient of the encoder output:
//   d_e2 = ELU'(e2) * conv4^T(dout)   on the 6 x 66 region the next step needs (zero outside
//                                     the image),
//   d_e1 = ELU'(e1) * conv2^T(d_e2)   on the tile,
//   dW4 += dout^T (x) e2,  dW2 += d_e2^T (x) e1,  dW0 += d_e1^T (x) in   (3x3 shifts, K = pixels),
//   db4 / db2 / db0 += column sums of dout / d_e2 / d_e1.
// Nothing but the weight-gradient partial slabs leaves the kernel: d_e2 and d_e1 live in
// LDS.  A workgroup walks tiles round-robin and keeps its 25 weight-gradient accumulator
// tiles (32 x 32) in registers; it writes one slab per weight (dvie_conv2d_wgrad layout,
// part[slab][o][t * cin + ci]) and per bias at the end.
// LDS images: dout [8 x 68 px][16 B]; e2, d_e2, e1 [6 x 66 px][64 B] and d_e1 [4 x 64][64 B]
// with 16-B chunk c of pixel p at (c ^ ((p >> 2) & 3)) (conflict-free row and transposed
// reads); in [6 x 66][48 B].  The conv-transpose products read A = packed data-gradient
// weights, B = the source image at the tap's shift (as the forward); the weight gradients
// read A = the output-gradient image and B = the input image at the tap's shift, both with
// ds_read_b64_tr_b16 transposed reads.
namespace dvie {

__device__ __forceinline__ bf16x8 hb_tr_pair_se(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// t + the sum of a fragment's 8 bf16 values, in fp32 (four v_dot2c_f32_bf16 against (1, 1))
__device__ __forceinline__ float sum8_bf16_se(const bf16x8 v, float t) {
  typedef __bf16 bf16x2_se __attribute__((ext_vector_type(2)));
  const i32x4 u = __builtin_bit_cast(i32x4, v);
  const bf16x2_se one = __builtin_bit_cast(bf16x2_se, 0x3F803F80);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int w = u[e];
    t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_se, w), one, t, false);
  }
  return t;
}

struct SbCfg {
  static constexpr int NW = 8, R = 4, TW = 64;
  static constexpr int DO_W = TW + 4, DO_H = R + 4;  // origin (-2, -2)
  static constexpr int E_W = TW + 2, E_H = R + 2;    // origin (-1, -1)
  static constexpr int DO_PC = (DO_H * DO_W + 63) / 64;
  static constexpr int E_PC = (E_H * E_W * 4 + 63) / 64;
  static constexpr int IN_PC = (E_H * E_W * 3 + 63) / 64;
  static constexpr int W4_PITCH = 5 * 32 + 16, W2_PITCH = 18 * 32 + 16;
  static constexpr int O_DO = 0, O_E2 = O_DO + DO_PC * 1024, O_E1 = O_E2 + E_PC * 1024, O_IN = O_E1 + E_PC * 1024;
  static constexpr int O_D2 = O_IN + IN_PC * 1024, O_D1 = O_D2 + E_H * E_W * 64, O_W4 = O_D1 + R * TW * 64;
  static constexpr int O_W2 = O_W4 + 32 * W4_PITCH, O_END = O_W2 + 32 * W2_PITCH;
  static constexpr int SMEM = O_END;
  static constexpr int PCS = DO_PC + 2 * E_PC + IN_PC;  // DMA pieces per tile
  static constexpr int PQ = (PCS + NW - 1) / NW;
};
static_assert(SbCfg::SMEM <= 163840, "segenc backward LDS");

// byte offset of 16-B chunk c of pixel p in a swizzled 64-B-pitch image
__device__ __forceinline__ int sw64(int p, int c) { return p * 64 + ((c ^ ((p >> 2) & 3)) << 4); }

// Phase 3 of the backward for one wave: its NBN 32-column blocks of weight-gradient GEMM
// GEMM (0: dW4 = dout^T (x) e2, 1: dW2 = d_e2^T (x) e1, 2: dW0 = d_e1^T (x) in) over the
// tile's 16 K-slices of 16 pixels.  A = the output-gradient image (rows o, 8 consecutive
// pixels per lane via two transposed reads), B = the input image at the tap's shift (columns
// n = t * cin + ci).  The lane's tap / channel of each block does not depend on the slice, so
// it is formed once; the next slice's fragments are read while the current slice's MFMAs run
// (one LDS round trip per slice instead of one per MFMA).
template <int GEMM, int NBN>
__device__ __forceinline__ void segenc_wg_phase(const char* smem, int nb0, f32x16 (&acc)[4], float& bsum, int g4, int qq,
                                                int pq) {
  typedef SbCfg C;
  constexpr int CIN = GEMM == 2 ? 24 : 32;
  int o0 = 16 * (g4 & 1) + 4 * pq;
  // (opaque per call: keeps the compiler from hoisting this phase's address arithmetic out of
  // the tile loop, where it would be held -- and spilled -- across the other phases)
  asm volatile("" : "+v"(o0));
  int tpo[NBN], cio[NBN];
#pragma unroll
  for (int j = 0; j < NBN; ++j) {
    const int n0 = 32 * (nb0 + j) + o0;
    int tp = n0 / CIN;
    cio[j] = n0 - tp * CIN;
    tp = tp < 9 ? tp : 8;  // columns past 9 cin: finite data, discarded
    tpo[j] = (tp / 3) * C::E_W + tp % 3;
  }
  // A row of the tile is 4 slices; within it the lane's fragments of slice k sit 16 pixels
  // past those of slice k - 1 in every image (the 64-B swizzle repeats every 4 pixels), so the
  // addresses are formed once per row and the slices read at immediate offsets
  constexpr int ASTEP = GEMM == 0 ? 16 * 16 : 16 * 64;
  constexpr int BSTEP = GEMM == 2 ? 16 * 48 : 16 * 64;
  struct Addr {
    const char *a0, *a1, *b0[NBN], *b1[NBN];
  };
  auto base = [&](int row) {
    Addr A;
    const int cc = 8 * (g4 >> 1) + qq;  // the lane's tile pixel in slice 0 of the row (+ 4 for the second read)
    const int pb = row * C::E_W + cc;   // the tile pixel in the 66-wide images, tap (0, 0)
    if constexpr (GEMM == 0) {  // dout rows o = o0 .. +3: rows past 7 read finite neighbours
      A.a0 = smem + C::O_DO + ((row + 2) * C::DO_W + cc + 2) * 16 + (o0 & 7) * 2;
      A.a1 = A.a0 + 4 * 16;
    } else if constexpr (GEMM == 1) {
      const int pe = pb + C::E_W + 1;
      A.a0 = smem + C::O_D2 + sw64(pe, o0 >> 3) + (o0 & 7) * 2;
      A.a1 = smem + C::O_D2 + sw64(pe + 4, o0 >> 3) + (o0 & 7) * 2;
    } else {
      const int P0 = 64 * row + cc;
      A.a0 = smem + C::O_D1 + sw64(P0, o0 >> 3) + (o0 & 7) * 2;
      A.a1 = smem + C::O_D1 + sw64(P0 + 4, o0 >> 3) + (o0 & 7) * 2;
    }
#pragma unroll
    for (int j = 0; j < NBN; ++j) {
      const int pe = pb + tpo[j];
      if constexpr (GEMM == 2) {
        A.b0[j] = smem + C::O_IN + pe * 48 + cio[j] * 2;
        A.b1[j] = A.b0[j] + 4 * 48;
      } else {
        constexpr int bb = GEMM == 0 ? C::O_E2 : C::O_E1;
        A.b0[j] = smem + bb + sw64(pe, cio[j] >> 3) + (cio[j] & 7) * 2;
        A.b1[j] = smem + bb + sw64(pe + 4, cio[j] >> 3) + (cio[j] & 7) * 2;
      }
    }
    return A;
  };
  auto fetch = [&](const Addr& A, int k, bf16x8& av, bf16x8 (&bv)[NBN]) {
    av = hb_tr_pair_se(A.a0 + k * ASTEP, A.a1 + k * ASTEP);
#pragma unroll
    for (int j = 0; j < NBN; ++j) bv[j] = hb_tr_pair_se(A.b0[j] + k * BSTEP, A.b1[j] + k * BSTEP);
  };
  auto step = [&](const bf16x8& av, const bf16x8 (&bv)[NBN]) {
#pragma unroll
    for (int j = 0; j < NBN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[j], acc[j], 0, 0, 0);
    // bias column sums from the A fragment: lane l holds 8 pixels of row l % 32 (the first
    // wave of each gemm sums; every wave does the VALU work, no branch splits the k-step)
    bsum = sum8_bf16_se(av, bsum);
  };
#pragma unroll 1
  for (int row = 0; row < 4; ++row) {
    const Addr A = base(row);
    bf16x8 a0, a1, b0[NBN], b1[NBN];
    fetch(A, 0, a0, b0);
    fetch(A, 1, a1, b1);
    step(a0, b0);
    fetch(A, 2, a0, b0);
    step(a1, b1);
    fetch(A, 3, a1, b1);
    step(a0, b0);
    step(a1, b1);
  }
}

__global__ __launch_bounds__(512) void segenc_bwd_kernel(const dvie_segenc_bwd_desc p, int tiles_x, int tiles_y,
                                                         int n_tiles, int dbg) {
  typedef SbCfg C;
  constexpr int NW = C::NW;
  dbg = DVIE_DBG(dbg);  // (timing-only ablations: a constant 0 outside -DDVIE_TIMING_DBG builds)
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5;
  const unsigned OOB = 0xFFFFFFF0u;

  // ---- data-gradient weights into LDS, once: w4d [32 ci][80 k], w2d [32 ci][288 k] ----
  for (int i = tid; i < 32 * 10; i += NW * 64) {
    const int r = i / 10, ch = i - r * 10;
    *(i32x4*)(smem + C::O_W4 + r * C::W4_PITCH + ch * 16) = *(const i32x4*)((const bf16_t*)p.w4d + r * p.kpad4 + ch * 8);
  }
  for (int i = tid; i < 32 * 36; i += NW * 64) {
    const int r = i / 36, ch = i - r * 36;
    *(i32x4*)(smem + C::O_W2 + r * C::W2_PITCH + ch * 16) = *(const i32x4*)((const bf16_t*)p.w2d + r * p.kpad2 + ch * 8);
  }

  // ---- DMA geometry: piece -> (image, slot) ----
  // images: 0 dout (1 chunk / px, origin -2), 1 e2 / 2 e1 (4 chunks, swizzled, origin -1), 3 in (3 chunks)
  int geo[C::PQ];
#pragma unroll
  for (int q = 0; q < C::PQ; ++q) {
    const int pc = wave + NW * q;
    int v = -1;
    if (pc < C::DO_PC) {
      const int px = pc * 64 + lane;
      if (px < C::DO_H * C::DO_W) v = (0 << 28) | ((px / C::DO_W) << 20) | ((px % C::DO_W) << 8);
    } else if (pc < C::DO_PC + 2 * C::E_PC) {
      const int img = pc < C::DO_PC + C::E_PC ? 1 : 2;
      const int slot = (pc - C::DO_PC - (img - 1) * C::E_PC) * 64 + lane, px = slot >> 2;
      const int src = (slot & 3) ^ ((px >> 2) & 3);
      if (px < C::E_H * C::E_W) v = (img << 28) | ((px / C::E_W) << 20) | ((px % C::E_W) << 8) | src;
    } else if (pc < C::PCS) {
      const int slot = (pc - C::DO_PC - 2 * C::E_PC) * 64 + lane, px = slot / 3;
      if (px < C::E_H * C::E_W) v = (3 << 28) | ((px / C::E_W) << 20) | ((px % C::E_W) << 8) | (slot - 3 * px);
    }
    geo[q] = v;
  }
  const unsigned long long npx = (unsigned long long)p.n * p.h * p.w;
  const __amdgpu_buffer_rsrc_t rs[4] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dout, 0, (int)((npx - 1) * p.dout_ld * 2ull + 16ull), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)p.e2, 0, (int)((npx - 1) * p.e2_ld * 2ull + 64ull), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)p.e1, 0, (int)((npx - 1) * p.e1_ld * 2ull + 64ull), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in, 0, (int)((npx - 1) * p.in_ld * 2ull + 48ull), 0x00020000)};
  const unsigned rows[4] = {(unsigned)p.dout_ld * 2u, (unsigned)p.e2_ld * 2u, (unsigned)p.e1_ld * 2u,
                            (unsigned)p.in_ld * 2u};

  // ---- weight-gradient accumulator tiles of this wave: (gemm, first N block, count) ----
  // waves 0-2: dW4 (M = 8 rows of 32, N = 288 = 9 blocks), 3-5: dW2 (9 blocks), 6-7: dW0 (7)
  const int gemm = wave < 3 ? 0 : wave < 6 ? 1 : 2;
  const int nb0 = gemm < 2 ? 3 * (wave - 3 * gemm) : (wave == 6 ? 0 : 4);
  const int nbn = gemm < 2 ? 3 : (wave == 6 ? 4 : 3);
  const int cin = gemm == 2 ? 24 : 32;
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  float bsum = 0.f;  // bias partial of the A rows (waves 0 / 3 / 6: dout / d_e2 / d_e1)

  // The next tile's four images are loaded into registers (10 x 16 B per lane) while this
  // tile's three phases run, and written to LDS at the next tile's start: the global-memory
  // latency of a tile's operands hides behind the previous tile's MFMAs (there is no room for a
  // second set of LDS images).
  i32x4 stg[C::PQ];
  auto tile_pos = [&](int t, int& n, int& y0, int& x0) {
    int tt = t;
    x0 = (tt % tiles_x) * C::TW;
    tt /= tiles_x;
    y0 = (tt % tiles_y) * C::R;
    n = tt / tiles_y;
  };
  auto load_tile = [&](int t) {
    int n, y0, x0;
    tile_pos(t, n, y0, x0);
#pragma unroll
    for (int q = 0; q < C::PQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::PCS) continue;  // (wave-uniform)
      int v = geo[q];
      asm volatile("" : "+v"(v));  // decoded per tile, not hoisted (and spilled) out of the loop
      const int img = pc < C::DO_PC ? 0 : pc < C::DO_PC + C::E_PC ? 1 : pc < C::DO_PC + 2 * C::E_PC ? 2 : 3;
      const int org = img == 0 ? 2 : 1;
      const int iy = y0 - org + ((v >> 20) & 0xFF), ix = x0 - org + ((v >> 8) & 0xFFF);
      const bool ok = v >= 0 && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
      const unsigned o = ok ? (unsigned)((n * p.h + iy) * p.w + ix) * rows[img] + (unsigned)(v & 15) * 16u : OOB;
      __amdgpu_buffer_rsrc_t r = img == 0 ? rs[0] : img == 1 ? rs[1] : img == 2 ? rs[2] : rs[3];
      stg[q] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < C::PQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::PCS) continue;
      const int img = pc < C::DO_PC ? 0 : pc < C::DO_PC + C::E_PC ? 1 : pc < C::DO_PC + 2 * C::E_PC ? 2 : 3;
      const int dst = img == 0 ? C::O_DO + pc * 1024
                               : img == 1 ? C::O_E2 + (pc - C::DO_PC) * 1024
                                          : img == 2 ? C::O_E1 + (pc - C::DO_PC - C::E_PC) * 1024
                                                     : C::O_IN + (pc - C::DO_PC - 2 * C::E_PC) * 1024;
      *(i32x4*)(smem + dst + lane * 16) = stg[q];
    }
  };
  if ((int)blockIdx.x < n_tiles && !(dbg & 64)) load_tile(blockIdx.x);

  for (int t = blockIdx.x; t < ((dbg & 32) ? 0 : n_tiles); t += gridDim.x) {
    int n, y0, x0;
    tile_pos(t, n, y0, x0);
    __syncthreads();  // the previous tile's reads of the images are done
    store_tile();
    __syncthreads();
    if (t + (int)gridDim.x < n_tiles && !(dbg & 8)) load_tile(t + gridDim.x);

    // the lane's fragment coordinates, opaque per tile: every phase forms its LDS addresses
    // from them inside the tile loop instead of the compiler hoisting all of them out of it
    // (where they were held, and spilled, across the phases)
    int lt = lane;
    asm volatile("" : "+v"(lt));
    const int r32 = lt & 31, hh = lt >> 5;
    const int g4 = lt >> 4, qq = (lt & 15) >> 2, pq = lt & 3;
    // ---- phase 1: d_e2 on the 6 x 66 region = ELU'(e2) * conv4^T(dout) ----
    // (dbg: timing-only ablation bits from DVIE_SEGENC_DBG, 0 in every real run: 1 / 2 / 4 skip
    // phase 1 / 2 / 3, 8 the tile loads, 16 the slab stores, 32 the whole tile loop, 64 the first tile's
    // loads)
    // A wave takes its blocks wave and wave + 8 together (13 blocks of 32 pixels): the weight
    // fragment of a k-step serves both, and the two MFMA chains interleave.
    auto p1_blocks = [&](auto nbt) {
      constexpr int NB = decltype(nbt)::value;
      constexpr int NPX = C::E_H * C::E_W;
      int q[NB], qc[NB];
      const char* B[NB];
      f32x16 a1[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        q[b] = (wave + NW * b) * 32 + r32;
        qc[b] = q[b] < NPX ? q[b] : NPX - 1;
        const int rr = qc[b] / C::E_W, cc = qc[b] - rr * C::E_W;
        B[b] = smem + C::O_DO + (rr * C::DO_W + cc) * 16;
#pragma unroll
        for (int e = 0; e < 16; ++e) a1[b][e] = 0.f;
      }
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const i32x4 a = *(const i32x4*)(smem + C::O_W4 + r32 * C::W4_PITCH + hh * 16 + s * 32);
        int kc = 2 * s + hh;
        kc = kc < 9 ? kc : 8;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const i32x4 bv = *(const i32x4*)(B[b] + ((kc / 3) * C::DO_W + kc % 3) * 16);
          a1[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, bv),
                                                          a1[b], 0, 0, 0);
        }
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int rr = qc[b] / C::E_W, cc = qc[b] - rr * C::E_W;
        const int gy = y0 - 1 + rr, gx = x0 - 1 + cc;
        const bool in = q[b] < NPX && (unsigned)gy < (unsigned)p.h && (unsigned)gx < (unsigned)p.w;
#pragma unroll
        for (int P = 0; P < 2; ++P) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1[b][8 * P + e]),
                                                             __float_as_uint(a1[b][8 * P + 4 + e]), false, false);
            v[e] = __uint_as_float(sw[0]);
            v[4 + e] = __uint_as_float(sw[1]);
          }
          const int ch = 2 * P + hh;  // 16-B chunk: channels 8 ch .. +7
          const i32x4 z = *(const i32x4*)(smem + C::O_E2 + sw64(qc[b], ch));
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float za = __uint_as_float(((uint32_t)z[e]) << 16), zb = __uint_as_float(((uint32_t)z[e]) & 0xffff0000u);
            o[e] = (int)se_pack(in ? v[2 * e] * act_dz(za, DVIE_ACT_ELU, 0.f) : 0.f,
                                in ? v[2 * e + 1] * act_dz(zb, DVIE_ACT_ELU, 0.f) : 0.f);
          }
          if (q[b] < NPX) *(i32x4*)(smem + C::O_D2 + sw64(q[b], ch)) = o;
        }
      }
    };
    static_assert((C::E_H * C::E_W + 31) / 32 <= 2 * NW, "phase 1: two blocks per wave");
    if (!(dbg & 1)) {
      if (wave + NW < (C::E_H * C::E_W + 31) / 32)
        p1_blocks(std::integral_constant<int, 2>());
      else
        p1_blocks(std::integral_constant<int, 1>());
    }
    __syncthreads();

    // ---- phase 2: d_e1 on the tile = ELU'(e1) * conv2^T(d_e2) ----
    if (!(dbg & 2)) {
      const int blk = wave;  // 8 blocks of 32 pixels
      const int q = blk * 32 + r32, rr = q >> 6, cc = q & 63;
      // (the K = 288 chain split over two accumulators: two independent MFMA chains; the
      // operands of k-step s + 2 are read while step s runs)
      f32x16 a1, a1b;
#pragma unroll
      for (int e = 0; e < 16; ++e) a1[e] = a1b[e] = 0.f;
      i32x4 ra[3], rb[3];
      auto ld2 = [&](int s, i32x4& a, i32x4& b) {
        a = *(const i32x4*)(smem + C::O_W2 + r32 * C::W2_PITCH + hh * 16 + s * 32);
        const int kc = 2 * s + hh, tp = kc >> 2, ck = kc & 3;
        const int pe = (rr + tp / 3) * C::E_W + cc + tp % 3;
        b = *(const i32x4*)(smem + C::O_D2 + sw64(pe, ck));
      };
      ld2(0, ra[0], rb[0]);
      ld2(1, ra[1], rb[1]);
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        if (s + 2 < 18) ld2(s + 2, ra[(s + 2) % 3], rb[(s + 2) % 3]);
        const bf16x8 av = __builtin_bit_cast(bf16x8, ra[s % 3]), bv = __builtin_bit_cast(bf16x8, rb[s % 3]);
        if (s & 1)
          a1b = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, a1b, 0, 0, 0);
        else
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, a1, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) a1[e] += a1b[e];
      const int gy = y0 + rr, gx = x0 + cc;
      const bool in = gy < p.h && gx < p.w;
      const int pe = (rr + 1) * C::E_W + cc + 1;
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1[8 * P + e]),
                                                           __float_as_uint(a1[8 * P + 4 + e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
        const int ch = 2 * P + hh;
        const i32x4 z = *(const i32x4*)(smem + C::O_E1 + sw64(pe, ch));
        i32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float za = __uint_as_float(((uint32_t)z[e]) << 16), zb = __uint_as_float(((uint32_t)z[e]) & 0xffff0000u);
          o[e] = (int)se_pack(in ? v[2 * e] * act_dz(za, DVIE_ACT_ELU, 0.f) : 0.f,
                              in ? v[2 * e + 1] * act_dz(zb, DVIE_ACT_ELU, 0.f) : 0.f);
        }
        *(i32x4*)(smem + C::O_D1 + sw64(q, ch)) = o;
      }
    }
    __syncthreads();

    // ---- phase 3: weight gradients over the tile's 256 pixels (K = pixels) ----
    if (dbg & 4) {
    } else if (gemm == 0)
      segenc_wg_phase<0, 3>(smem, nb0, acc, bsum, g4, qq, pq);
    else if (gemm == 1)
      segenc_wg_phase<1, 3>(smem, nb0, acc, bsum, g4, qq, pq);
    else if (nbn == 4)
      segenc_wg_phase<2, 4>(smem, nb0, acc, bsum, g4, qq, pq);
    else
      segenc_wg_phase<2, 3>(smem, nb0, acc, bsum, g4, qq, pq);
    // the next tile's images: issued after this tile's phases, so the 10 x 16 B per lane they
    // land in are not held across the phases (whose MFMAs need the registers for operand
    // pipelining); their latency is exposed once per tile at the store above
  }

  // ---- this workgroup's slabs ----
  const int slab = blockIdx.x;
  if (!(dbg & 16)) {
    float* out = gemm == 0 ? p.dw4 : gemm == 1 ? p.dw2 : p.dw0;
    const int cout = gemm == 0 ? 8 : 32, kw = 9 * cin;
    out += (long long)slab * cout * kw;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= nbn) break;
      const int n = 32 * (nb0 + j) + (lane & 31);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int o = 8 * i + 4 * hh + e;
          if (o < cout && n < kw) out[o * kw + n] = acc[j][4 * i + e];
        }
    }
  }
  // bias partials: lanes l and l + 32 hold the two 8-pixel halves of row l % 32 (dout's
  // rows 8..31 are copies of rows 0..7)
  const float bt = bsum + __shfl_xor(bsum, 32, 64);
  if (wave == 0 && lane < 8) p.db4[slab * 8 + lane] = bt;
  if (wave == 3 && lane < 32) p.db2[slab * 32 + lane] = bt;
  if (wave == 6 && lane < 32) p.db0[slab * 32 + lane] = bt;
}

}  // namespace dvie

extern "C" int dvie_segenc_bwd(const dvie_segenc_bwd_desc* d, void* stream) {
  using namespace dvie;
  DVIE_CHECK_ARG(d && d->dout && d->e2 && d->e1 && d->in && d->w4d && d->w2d, "segenc_bwd: null pointer");
  DVIE_CHECK_ARG(d->dw4 && d->dw2 && d->dw0 && d->db4 && d->db2 && d->db0, "segenc_bwd: null slab");
  DVIE_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->slabs > 0, "segenc_bwd: shape");
  DVIE_CHECK_ARG(d->dout_ld >= 8 && d->e2_ld >= 32 && d->e1_ld >= 32 && d->in_ld >= 24, "segenc_bwd: leading dims");
  DVIE_CHECK_ARG(d->kpad4 >= 80 && d->kpad2 >= 288, "segenc_bwd: kpad");
  const unsigned long long npx = (unsigned long long)d->n * d->h * d->w;
  const long long ld = std::max(std::max(d->dout_ld, d->e2_ld), std::max(d->e1_ld, d->in_ld));
  DVIE_CHECK_ARG(npx * (unsigned long long)ld * 2ull < 0xFFFFFF00ull && npx < (1ull << 31),
                 "segenc_bwd: maps exceed the 32-bit buffer range");
  const int tiles_x = (d->w + 63) / 64, tiles_y = (d->h + 3) / 4;
  const long long nt = (long long)tiles_x * tiles_y * d->n;
  DVIE_CHECK_ARG(nt < (1LL << 30), "segenc_bwd: too many tiles");
  int dbg = 0;  // DVIE_SEGENC_DBG: timing-only ablations (tools/segenc_micro.py), -DDVIE_TIMING_DBG builds only
#ifdef DVIE_TIMING_DBG
  if (const char* e = getenv("DVIE_SEGENC_DBG")) dbg = atoi(e);
#endif
  DVIE_LAUNCH(segenc_bwd_kernel, dim3(d->slabs), dim3(512), 0, (hipStream_t)stream, *d, tiles_x, tiles_y,
                     (int)nt, dbg);
  DVIE_RETURN_LAUNCH();
}
