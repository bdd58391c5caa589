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
// Each wave takes 32-pixel blocks round-robin; `epi(q, lane_channels, v[8])` consumes the
// 8 consecutive channels 16 P + 8 hh .. +7 (P = 0, 1) of pixel q.
template <int KS, int CPT, int RW, int SP, int WP, typename Epi>
__device__ __forceinline__ void se_stage(const char* Wl, int wrows, const char* Src, int npx, int wave, int lane,
                                         Epi&& epi) {
  constexpr int SW = RW + 2;
  constexpr int KC = 9 * CPT;
  const int r32 = lane & 31, hh = lane >> 5;
  const char* Wa = Wl + (r32 < wrows ? r32 : r32 & (wrows - 1)) * WP + hh * 16;
  const int nblk = (npx + 31) / 32;
  for (int blk = wave; blk < nblk; blk += SeCfg::NW) {
    const int q = blk * 32 + r32;
    const int qc = q < npx ? q : npx - 1;  // (pad lanes read a valid pixel, results dropped)
    const int r = qc / RW, c = qc - r * RW;
    const char* B = Src + (r * SW + c) * SP;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const i32x4 a = *(const i32x4*)(Wa + s * 32);
      int kc = 2 * s + hh;
      kc = kc < KC ? kc : KC - 1;  // zero-weight padding chunk: any finite source
      const int t = kc / CPT, cc = kc - t * CPT;
      const i32x4 b = *(const i32x4*)(B + ((t / 3) * SW + t % 3) * SP + cc * 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                    0, 0, 0);
    }
    float v[2][8];
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[8 * P + e]),
                                                         __float_as_uint(acc[8 * P + 4 + e]), false, false);
        v[P][e] = __uint_as_float(sw[0]);
        v[P][4 + e] = __uint_as_float(sw[1]);
      }
    if (q < npx) epi(q / RW, q % RW, v);
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

  const int G = gridDim.x;
  for (int t = blockIdx.x; t < n_tiles; t += G) {
    int tt = t;
    const int x0 = (tt % tiles_x) * C::TW;
    tt /= tiles_x;
    const int y0 = (tt % tiles_y) * C::R;
    const int n = tt / tiles_y;
    // previous tile's readers are done with every image (and the weights have landed)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < IQ; ++q) {
      const int pc = wave + NW * q;
      if (pc >= C::IN_PC) continue;  // (wave-uniform)
      const int v = igeo[q];
      const int iy = y0 - 3 + ((v >> 16) & 0xFF), ix = x0 - 3 + ((v >> 4) & 0xFFF);
      const bool ok = v >= 0 && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
      const unsigned o = ok ? (unsigned)((n * p.h + iy) * p.w + ix) * irow + (unsigned)(v & 15) * 16u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_ptr_se)(smem + C::O_IN + pc * 1024), 16, o, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

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
              const float a = in ? act_fwd(v[P][2 * e] + p.b0[co + 2 * e], DVIE_ACT_ELU, 0.f) : 0.f;
              const float b = in ? act_fwd(v[P][2 * e + 1] + p.b0[co + 2 * e + 1], DVIE_ACT_ELU, 0.f) : 0.f;
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
              const float a = in ? act_fwd(v[P][2 * e] + p.b2[co + 2 * e], DVIE_ACT_ELU, 0.f) : 0.f;
              const float b = in ? act_fwd(v[P][2 * e + 1] + p.b2[co + 2 * e + 1], DVIE_ACT_ELU, 0.f) : 0.f;
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
          for (int e = 0; e < 4; ++e) o[e] = (int)se_pack(v[0][2 * e] + p.b4[2 * e], v[0][2 * e + 1] + p.b4[2 * e + 1]);
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
  hipLaunchKernelGGL(segenc_fwd_kernel, dim3(grid), dim3(512), 0, (hipStream_t)stream, *d, tiles_x, tiles_y, (int)nt);
  DVIE_RETURN_LAUNCH();
}
