// Convolution kernels for gfx950 (MI355X, CDNA4).
//
// (the implicit-GEMM forward / data-gradient kernel lives in conv_fwd.hip)
//
// wgrad: per tap, dW[co][ci] = sum_pix g[pix][co] * x[pix+tap][ci], split over pixel
//   chunks into fp32 partial slabs (no atomics, deterministic), reduced by wreduce into
//   the OIHW fp32 parameter gradient.  bf16 operands reach MFMA through
//   ds_read_b64_tr_b16 transposed reads of [pixel][channel] LDS images.
//
// Reference ops replaced: nn.Conv2d forward / backward of nets/HRNet.py (all 77 convs)
// and nets/vgg.py:11-54 (VGG19 features).
#include <cxxabi.h>
#include <dlfcn.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "common.h"

namespace dvie {

static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

// launch trace (dvie_trace_kernels): the host stubs of the kernels this thread launched
thread_local bool g_trace_on = false;
static thread_local std::vector<const void*> g_trace;
static thread_local std::string g_trace_text;
void trace_launch(const void* fn) {
  if (g_trace.size() < 4096) g_trace.push_back(fn);
}

static std::string kernel_name(const void* fn) {
  const char* m = hipKernelNameRefByPtr(fn, nullptr);
  Dl_info info;
  if (!m && dladdr(fn, &info) && info.dli_sname) m = info.dli_sname;
  if (!m) {
    char b[32];
    snprintf(b, sizeof(b), "%p", fn);
    return b;
  }
  int st = 0;
  char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
  std::string out = (st == 0 && d) ? d : m;
  free(d);
  return out;
}

// ----------------------------------------------------------------------------------
// weight gradient
// ----------------------------------------------------------------------------------
// bf16 image: [64 pixels][64 channels] = 128-byte rows, 32-byte blocks XOR-swizzled so
// that the 8 rows read by a half-wave's ds_read_b64_tr_b16 cover all 64 banks.
__device__ __forceinline__ int wsw_f(int row) { return ((row >> 1) & 1) | ((row >> 2) & 2); }
__device__ __forceinline__ int wswz(int row, int blk) { return row * 128 + ((blk ^ wsw_f(row)) << 5); }

template <typename T>
struct WgCfg;
template <>
struct WgCfg<bf16_t> {
  static constexpr int BKP = 64;      // pixels per stage
  static constexpr int ROWB = 128;    // bytes per LDS row (64 channels)
  static constexpr int CHR = 8;       // 16-byte chunks per row
};
template <>
struct WgCfg<float> {
  static constexpr int BKP = 32;
  static constexpr int ROWB = 320;    // 64 floats + 16 floats pad
  static constexpr int CHR = 16;
};

struct PixCursor {
  int n, oy, ox;  // current pixel of this staged row
  bool valid;
};

template <typename T>
__global__ __launch_bounds__(256) void wgrad_kernel(const dvie_wgrad_desc p, long long chunk) {
  constexpr int BM = 64, BN = 64;
  constexpr int ES = sizeof(T);
  constexpr int VEC = 16 / ES;
  constexpr int BKP = WgCfg<T>::BKP;
  constexpr int ROWB = WgCfg<T>::ROWB;
  constexpr int CHR = WgCfg<T>::CHR;
  constexpr int IT = BKP * CHR / 256;  // 16B chunks per thread per operand = 2
  constexpr int RSTEP = 256 / CHR;     // rows advanced between a thread's chunks
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BKP * ROWB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int split = blockIdx.x;
  const int ntn = (p.c + BN - 1) / BN;
  const int m0 = (blockIdx.y / ntn) * BM;
  const int n0 = (blockIdx.y % ntn) * BN;
  const int tap = blockIdx.z;
  const int ti = tap / p.tw, tj = tap - (tap / p.tw) * p.tw;
  const int dy = p.dy0 + ti * p.ddy, dx = p.dx0 + tj * p.ddx;
  const int hw = p.oh * p.ow;
  const long long npix = (long long)p.n * hw;
  const long long pbeg = (long long)split * chunk;
  const long long pend = pbeg + chunk < npix ? pbeg + chunk : npix;
  const int nk = pbeg < pend ? (int)((pend - pbeg + BKP - 1) / BKP) : 0;
  const char* __restrict__ gg = (const char*)p.g;
  const char* __restrict__ xg = (const char*)p.x;

  const int cc = tid % CHR;        // chunk (channel group) within the row
  const int row0 = tid / CHR;      // first staged row
  // running pixel cursors for rows row0 + i*RSTEP
  long long pix[IT];
  int cn[IT], coy[IT], cox[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    pix[i] = pbeg + row0 + i * RSTEP;
    const long long q = pix[i] < npix ? pix[i] : 0;
    cn[i] = (int)(q / hw);
    const int r = (int)(q - (long long)cn[i] * hw);
    coy[i] = r / p.ow;
    cox[i] = r - coy[i] * p.ow;
  }

  i32x4 ra[IT], rb[IT];
  const bool a_ok = (m0 + cc * VEC) < p.cout;
  const bool b_ok = (n0 + cc * VEC) < p.c;
  auto load_stage = [&]() {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const bool pv = pix[i] < pend;
      if (pv && a_ok) {
        const long long off = (pix[i] * p.g_ld + m0 + cc * VEC) * ES;
        ra[i] = *(const i32x4*)(gg + off);
      } else {
        ra[i] = i32x4{0, 0, 0, 0};
      }
      const int iy = coy[i] * p.sy + dy, ix = cox[i] * p.sx + dx;
      if (pv && b_ok && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw) {
        const long long off = ((((long long)cn[i] * p.ih + iy) * p.iw + ix) * p.x_ld + n0 + cc * VEC) * ES;
        rb[i] = *(const i32x4*)(xg + off);
      } else {
        rb[i] = i32x4{0, 0, 0, 0};
      }
      // advance this row's pixel by BKP
      pix[i] += BKP;
      cox[i] += BKP;
      while (cox[i] >= p.ow) {
        cox[i] -= p.ow;
        if (++coy[i] >= p.oh) {
          coy[i] = 0;
          ++cn[i];
        }
      }
    }
  };
  auto store_stage = [&](int buf) {
    char* As = smem + buf * 2 * BKP * ROWB;
    char* Bs = As + BKP * ROWB;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int row = row0 + i * RSTEP;
      int off;
      if constexpr (sizeof(T) == 2)
        off = wswz(row, cc >> 1) + ((cc & 1) << 4);
      else
        off = row * ROWB + cc * 16;
      *(i32x4*)(As + off) = ra[i];
      *(i32x4*)(Bs + off) = rb[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load_stage();
    store_stage(0);
  }
  __syncthreads();
  const int g = lane >> 4, r16 = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage();
    const char* As = smem + cur * 2 * BKP * ROWB;
    const char* Bs = As + BKP * ROWB;
    if constexpr (sizeof(T) == 2) {
      const int q = r16 >> 2, pp = r16 & 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        i32x4 af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int cb = (wm * 32 + 16 * i) >> 4;  // 16-channel block
          const int rowa = 32 * s + 8 * g + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(As + wswz(rowa, cb) + 8 * pp));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(As + wswz(rowa + 4, cb) + 8 * pp));
          af[i] = i32x4{(int)((uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16)),
                        (int)((uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16)),
                        (int)((uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16)),
                        (int)((uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16))};
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int cb = (wn * 32 + 16 * j) >> 4;
          const int rowb = 32 * s + 8 * g + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Bs + wswz(rowb, cb) + 8 * pp));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Bs + wswz(rowb + 4, cb) + 8 * pp));
          bf[j] = i32x4{(int)((uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16)),
                        (int)((uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16)),
                        (int)((uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16)),
                        (int)((uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16))};
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                __builtin_bit_cast(bf16x8, bf[j]), acc[i][j], 0, 0,
                                                                0);
      }
    } else {
      const float* Af = (const float*)As;
      const float* Bf = (const float*)Bs;
      constexpr int RF = ROWB / 4;
#pragma unroll
      for (int k = 0; k < BKP; k += 4) {
        float a0 = Af[(k + g) * RF + wm * 32 + r16];
        float a1 = Af[(k + g) * RF + wm * 32 + 16 + r16];
        float b0 = Bf[(k + g) * RF + wn * 32 + r16];
        float b1 = Bf[(k + g) * RF + wn * 32 + 16 + r16];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_stage(cur ^ 1);
    __syncthreads();
  }

  // partial slab: ws[split][co][tap*c + ci]
  const long long kw = (long long)p.th * p.tw * p.c;
  float* __restrict__ out = p.ws + (long long)split * p.cout * kw;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = n0 + wn * 32 + 16 * j + r16;
      if (ci >= p.c) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = m0 + wm * 32 + 16 * i + 4 * g + e;
        if (co < p.cout) out[(long long)co * kw + (long long)tap * p.c + ci] = acc[i][j][e];
      }
    }
}

// QB float4 columns x SL split-lanes per block (QB * SL = 256): every thread streams every
// SL-th slab of its 16-byte column (coalesced rows per slab), fp64 accumulation, LDS fold,
// scatter into the OIHW gradient.  Wide reductions (weights) use 32 x 8; narrow ones with
// many slabs (bias column sums: cout/4 columns, thousands of partials) 4 x 64.
template <int QB, int SL>
__device__ __forceinline__ void wreduce_block(const dvie_wreduce_desc& p, int bx) {
  static_assert(QB * SL == 256, "block shape");
  __shared__ double red[SL][QB][4];
  const int tid = threadIdx.x;
  const int ql = tid % QB, sl = tid / QB;
  const int taps = p.kh_n * p.kw_n;
  const long long total4 = (long long)(p.ws_rows - p.co_off) * p.ws_k / 4;  // scanned (padded) rows
  const long long slab = (long long)p.ws_rows * p.ws_k;
  const long long q = (long long)bx * QB + ql;
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  if (q < total4) {
    const float* src = p.ws + (long long)p.co_off * p.ws_k + q * 4;
    // four slabs' loads issued before their adds: one memory latency per four slabs (a plain
    // loop waits for each load before issuing the next)
    int k = sl;
    for (; k + 3 * SL < p.splits; k += 4 * SL) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const f32x4*)(src + (k + u * SL) * slab);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a0 += v[u][0];
        a1 += v[u][1];
        a2 += v[u][2];
        a3 += v[u][3];
      }
    }
    for (; k < p.splits; k += SL) {
      const f32x4 v = *(const f32x4*)(src + k * slab);
      a0 += v[0];
      a1 += v[1];
      a2 += v[2];
      a3 += v[3];
    }
  }
  red[sl][ql][0] = a0;
  red[sl][ql][1] = a1;
  red[sl][ql][2] = a2;
  red[sl][ql][3] = a3;
  __syncthreads();
  if (tid < QB * 4) {
    const int qq = tid >> 2, e = tid & 3;
    const long long f = ((long long)bx * QB + qq) * 4 + e;
    if (f < total4 * 4) {
      double s = 0;
      for (int k = 0; k < SL; ++k) s += red[k][qq][e];
      const int co = (int)(f / p.ws_k);
      const int rem = (int)(f - (long long)co * p.ws_k);
      const int t = rem / p.c, j = rem - (rem / p.c) * p.c;
      const int ci = p.cmap ? p.cmap[j] : j;
      if (co < p.cout_p && ci >= 0 && ci < p.cin_p && t < taps) {
        const long long o = (((long long)co * p.cin_p + ci) * p.kh_n + t / p.kw_n) * p.kw_n + t % p.kw_n;
        float v = (float)s;
        if (p.beta) v += p.dw[o];
        p.dw[o] = v;
      }
    }
  }
}

template <int QB, int SL>
__global__ __launch_bounds__(256) void wreduce_kernel(const dvie_wreduce_desc p) {
  wreduce_block<QB, SL>(p, blockIdx.x);
}

// up to WRM reductions in one launch: descriptor i owns blocks [blk0[i], blk0[i + 1])
constexpr int WRM = 16;
struct WreduceMulti {
  dvie_wreduce_desc d[WRM];
  int blk0[WRM + 1];
  int n;
};

__global__ __launch_bounds__(256) void wreduce_multi_kernel(const WreduceMulti m) {
  int i = 0;
  while (i + 1 < m.n && (int)blockIdx.x >= m.blk0[i + 1]) ++i;  // (uniform per block)
  wreduce_block<32, 8>(m.d[i], (int)blockIdx.x - m.blk0[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const dvie_colsum_desc p, long long chunk) {
  __shared__ float red[256 * 4];
  const int cq = p.c / 4;
  const int nrl = cq >= 256 ? 1 : 256 / cq;
  const int tid = threadIdx.x;
  const long long rbeg = (long long)blockIdx.x * chunk;
  const long long rend = rbeg + chunk < p.rows ? rbeg + chunk : p.rows;
  for (int qb = 0; qb < cq; qb += 256 / nrl) {
    const int q = qb + tid % (256 / nrl);
    const int rl = tid / (256 / nrl);
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q < cq && rl < nrl) {
      // four independent row streams per thread: four loads in flight per iteration
      const T* g = (const T*)p.g + 4 * q;
      f32x4 s1 = s, s2 = s, s3 = s;
      long long r = rbeg + rl;
      for (; r + 3 * nrl < rend; r += 4 * nrl) {
        const f32x4 a = V4<T>::load(g + r * p.g_ld), b = V4<T>::load(g + (r + nrl) * p.g_ld);
        const f32x4 c = V4<T>::load(g + (r + 2 * nrl) * p.g_ld), d = V4<T>::load(g + (r + 3 * nrl) * p.g_ld);
        s += a;
        s1 += b;
        s2 += c;
        s3 += d;
      }
      for (; r < rend; r += nrl) s += V4<T>::load(g + r * p.g_ld);
      s += (s1 + s2) + s3;
    }
    for (int e = 0; e < 4; ++e) red[tid * 4 + e] = s[e];
    __syncthreads();
    if (tid < 256 / nrl && qb + tid < cq) {
      f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < nrl; ++k)
        for (int e = 0; e < 4; ++e) t[e] += red[(k * (256 / nrl) + tid) * 4 + e];
      for (int e = 0; e < 4; ++e) p.ws[(long long)blockIdx.x * p.c + 4 * (qb + tid) + e] = t[e];
    }
    __syncthreads();
  }
}

// Flat grid: block b belongs to the last descriptor whose blk0 <= b (uniform binary search).
// Three block kinds, a pure function of the descriptor (pack_kind; engine.py pack_blocks
// mirrors it):
//   ROW  (mode 0, kpad >= 64): one packed row; its source row w[co][:][:][:] is contiguous,
//        so it is staged in LDS by coalesced loads and the row written 4 elements per thread.
//   TILE (mode 1, kpad >= 64): 8 packed rows (source channels) x 64 columns (output
//        channels); the source block w[co0 .. +64][ci of the 8 rows][taps] is staged in LDS
//        (contiguous per co), then every (row, tap) writes 64 consecutive columns.
//   ELEM (the rest: biases, tiny layers): 1024 elements, 4 per thread.
// The element-wise form alone gathered every source value with a 36 B (mode 0) or cin * 36 B
// (mode 1) stride: 0.27 ms per step for ~40 MB of weights.
enum { PACK_ELEM = 0, PACK_ROW = 1, PACK_TILE = 2 };
constexpr int PACK_LDS = 8192;  // floats
constexpr int PACK_TR = 8, PACK_TC = 64;

__host__ __device__ inline int pack_kind(const dvie_pack_desc& d) {
  if (d.kpad < 64 || d.kpad % 4 != 0) return PACK_ELEM;
  if (d.mode == 0 && d.cin_s * d.kh_s * d.kw_s <= PACK_LDS) return PACK_ROW;
  if (d.mode == 1 && d.kh_s * d.kw_s <= 16 && d.c % 4 == 0) return PACK_TILE;
  return PACK_ELEM;
}

__device__ __forceinline__ void pack_store4(const dvie_pack_desc& p, long long e, const float* v) {
  if (p.dtype == DVIE_BF16) {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)((bf16_t*)p.dst + e) = u;
  } else {
    *(f32x4*)((float*)p.dst + e) = f32x4{v[0], v[1], v[2], v[3]};
  }
}

__global__ __launch_bounds__(256) void pack_kernel(const dvie_pack_desc* __restrict__ descs, int n) {
  __shared__ float lds[PACK_LDS];
  int lo = 0, hi = n - 1;
  const int b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].blk0 <= b)
      lo = mid;
    else
      hi = mid - 1;
  }
  const dvie_pack_desc p = descs[lo];
  const int lb = b - p.blk0;
  const int ntap = p.th * p.tw, tid = threadIdx.x;
  const int kind = pack_kind(p);

  if (kind == PACK_ROW) {
    // packed row r = output channel co: dst[r][t c + j] = w[r][cmap[j]][kh(t)][kw(t)]
    const int r = lb, L = p.cin_s * p.kh_s * p.kw_s;
    const bool live = r < p.cout_s;
    for (int i = tid; i < L; i += 256) lds[i] = live ? p.src[(long long)r * L + i] : 0.f;
    __syncthreads();
    for (int k0 = 4 * tid; k0 < p.kpad; k0 += 1024) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = k0 + q, t = k / p.c, j = k - t * p.c;
        v[q] = 0.f;
        if (live && t < ntap) {
          const int ci = p.cmap ? p.cmap[j] : j;
          const int kh = p.kh0 + (t / p.tw) * p.dkh, kw = p.kw0 + (t % p.tw) * p.dkw;
          if (ci >= 0 && ci < p.cin_s && kh >= 0 && kh < p.kh_s && kw >= 0 && kw < p.kw_s)
            v[q] = lds[(ci * p.kh_s + kh) * p.kw_s + kw];
        }
      }
      pack_store4(p, (long long)r * p.kpad + k0, v);
    }
    return;
  }
  if (kind == PACK_TILE) {
    // rows r0 .. r0+7 (source channels cmap[r]), columns j0 .. j0+63 (output channels) of
    // every tap: dst[r][t c + j] = w[j][cmap[r]][kh(t)][kw(t)]
    const int ncb = (p.c + PACK_TC - 1) / PACK_TC;
    const int r0 = (lb / ncb) * PACK_TR, j0 = (lb % ncb) * PACK_TC;
    const int T = p.kh_s * p.kw_s;
    for (int i = tid; i < PACK_TC * PACK_TR * T; i += 256) {  // lds[jj][k][tap], tap fastest
      const int jj = i / (PACK_TR * T), rem = i - jj * (PACK_TR * T), k = rem / T, tp = rem - k * T;
      const int co = j0 + jj, r = r0 + k;
      const int ci = r < p.rows ? (p.cmap ? p.cmap[r] : r) : -1;
      lds[i] = (co < p.cout_s && ci >= 0 && ci < p.cin_s) ? p.src[((long long)co * p.cin_s + ci) * T + tp] : 0.f;
    }
    __syncthreads();
    const int nq = PACK_TC / 4;  // 4 consecutive columns per thread
    for (int i = tid; i < PACK_TR * ntap * nq; i += 256) {
      const int k = i / (ntap * nq), rem = i - k * (ntap * nq), t = rem / nq, jq = rem - t * nq;
      const int r = r0 + k, j = j0 + 4 * jq;
      if (r >= p.rows || j >= p.c) continue;
      const int kh = p.kh0 + (t / p.tw) * p.dkh, kw = p.kw0 + (t % p.tw) * p.dkw;
      const bool tap_ok = kh >= 0 && kh < p.kh_s && kw >= 0 && kw < p.kw_s;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = tap_ok ? lds[((j - j0 + q) * PACK_TR + k) * T + kh * p.kw_s + kw] : 0.f;
      pack_store4(p, (long long)r * p.kpad + t * p.c + j, v);
    }
    if (j0 == 0) {  // the K padding [ntap c, kpad) of these rows
      const int pad = p.kpad - ntap * p.c;
      for (int i = tid; i < PACK_TR * (pad / 4); i += 256) {
        const int k = i / (pad / 4), q4 = i - k * (pad / 4);
        const float z[4] = {0.f, 0.f, 0.f, 0.f};
        if (r0 + k < p.rows) pack_store4(p, (long long)(r0 + k) * p.kpad + ntap * p.c + 4 * q4, z);
      }
    }
    return;
  }
  // ELEM
  const long long total = (long long)p.rows * p.kpad;
  const long long e0 = ((long long)lb * 256 + tid) * 4;
  if (e0 >= total) return;
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long e = e0 + q;
    v[q] = 0.f;
    if (e >= total) continue;
    const int r = (int)(e / p.kpad);
    const int k = (int)(e - (long long)r * p.kpad);
    const int t = k / p.c;
    const int j = k - t * p.c;
    if (t < ntap) {
      int co, ci;
      if (p.mode == 0) {
        co = r;
        ci = p.cmap ? p.cmap[j] : j;
      } else {
        co = j;
        ci = p.cmap ? p.cmap[r] : r;
      }
      const int kh = p.kh0 + (t / p.tw) * p.dkh;
      const int kw = p.kw0 + (t % p.tw) * p.dkw;
      if (co < p.cout_s && ci >= 0 && ci < p.cin_s && kh >= 0 && kh < p.kh_s && kw >= 0 && kw < p.kw_s)
        v[q] = p.src[(((long long)co * p.cin_s + ci) * p.kh_s + kh) * p.kw_s + kw];
    }
  }
  if (e0 + 4 <= total && p.kpad % 4 == 0) {  // four of one row, aligned
    pack_store4(p, e0, v);
  } else if (p.dtype == DVIE_BF16) {
    for (int q = 0; q < 4; ++q)
      if (e0 + q < total) ((bf16_t*)p.dst)[e0 + q] = f2bf(v[q]);
  } else {
    for (int q = 0; q < 4; ++q)
      if (e0 + q < total) ((float*)p.dst)[e0 + q] = v[q];
  }
}

}  // namespace dvie

using namespace dvie;

namespace dvie {
int wgrad_halo_splits(const dvie_wgrad_desc& p);  // wgrad_halo.hip
int wgrad_halo_slabs(const dvie_wgrad_desc& p);
int wgrad_halo_bias_slabs(const dvie_wgrad_desc& p);
bool wgrad_halo_launch(const dvie_wgrad_desc& p, hipStream_t s);
}  // namespace dvie

extern "C" {

int dvie_wgrad_splits_hint(const dvie_wgrad_desc* d) { return d ? wgrad_halo_splits(*d) : 0; }

int dvie_wgrad_slabs(const dvie_wgrad_desc* d) { return d ? wgrad_halo_slabs(*d) : 0; }

// bias column sums as a pass of their own, for launches the halo kernels do not take
static int colsum_bias_splits(const dvie_wgrad_desc& d) {
  const long long npix = (long long)d.n * d.oh * d.ow;
  const long long s = npix / 512;  // >= 8 blocks per CU at full resolution
  return (int)(s < 1 ? 1 : (s > 2048 ? 2048 : s));
}

static void launch_bias_colsum(const dvie_wgrad_desc& d, hipStream_t s) {
  dvie_colsum_desc c{};
  c.g = d.g;
  c.ws = d.bws;
  c.g_ld = d.g_ld;
  c.rows = (long long)d.n * d.oh * d.ow;
  c.c = d.cout;
  c.splits = colsum_bias_splits(d);
  c.dtype = d.dtype;
  const long long chunk = (c.rows + c.splits - 1) / c.splits;
  if (d.dtype == DVIE_BF16)
    DVIE_LAUNCH(colsum_kernel<bf16_t>, dim3(c.splits), dim3(256), 0, s, c, chunk);
  else
    DVIE_LAUNCH(colsum_kernel<float>, dim3(c.splits), dim3(256), 0, s, c, chunk);
}

int dvie_wgrad_bias_slabs(const dvie_wgrad_desc* d) {
  if (!d) return 0;
  const int h = wgrad_halo_bias_slabs(*d);
  return h > 0 ? h : colsum_bias_splits(*d);
}

int dvie_conv2d_wgrad(const dvie_wgrad_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->g && d->x && d->ws, "wgrad: null pointer");
  const int vec = d->dtype == DVIE_BF16 ? 8 : 4;
  DVIE_CHECK_ARG(d->c % vec == 0 && d->g_ld % vec == 0 && d->x_ld % vec == 0,
                 "wgrad: channel alignment c=%d g_ld=%lld x_ld=%lld", d->c, d->g_ld, d->x_ld);
  DVIE_CHECK_ARG(d->splits >= 1, "wgrad: splits");
  const long long npix = (long long)d->n * d->oh * d->ow;
  const int bkp = d->dtype == DVIE_BF16 ? 64 : 32;
  long long chunk = (npix + d->splits - 1) / d->splits;
  chunk = (chunk + bkp - 1) / bkp * bkp;
  dim3 grid((unsigned)d->splits, (unsigned)(((d->cout + 63) / 64) * ((d->c + 63) / 64)), (unsigned)(d->th * d->tw));
  hipStream_t s = (hipStream_t)stream;
  if (d->bws) DVIE_CHECK_ARG(d->cout % 4 == 0 && d->cout <= 4096 && d->g_ld % 4 == 0, "wgrad: bias partials (cout=%d)", d->cout);
  if (wgrad_halo_launch(*d, s)) DVIE_RETURN_LAUNCH();  // (bias sums fused when bws is set)
  DVIE_CHECK_ARG(d->ws_taps == 0, "wgrad: a shared-slab phase launch (ws_taps=%d) needs the halo kernel "
                 "(bf16, stride 1 over the phase view, ow %% 64 == 0)", d->ws_taps);
  if (d->dtype == DVIE_BF16)
    DVIE_LAUNCH(wgrad_kernel<bf16_t>, grid, dim3(256), 0, s, *d, chunk);
  else
    DVIE_LAUNCH(wgrad_kernel<float>, grid, dim3(256), 0, s, *d, chunk);
  if (d->bws) launch_bias_colsum(*d, s);
  DVIE_RETURN_LAUNCH();
}

static int wreduce_check(const dvie_wreduce_desc* d);

int dvie_wgrad_reduce(const dvie_wreduce_desc* d, void* stream) {
  const int rc = wreduce_check(d);
  if (rc != DVIE_OK) return rc;
  const long long total4 = (long long)(d->ws_rows - d->co_off) * d->ws_k / 4;
  if (total4 < 1) return DVIE_OK;
  if (total4 < 2048 && d->splits >= 256)
    DVIE_LAUNCH((wreduce_kernel<4, 64>), dim3((unsigned)((total4 + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       *d);
  else
    DVIE_LAUNCH((wreduce_kernel<32, 8>), dim3((unsigned)((total4 + 31) / 32)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

static int wreduce_check(const dvie_wreduce_desc* d) {
  DVIE_CHECK_ARG(d && d->ws && d->dw, "wreduce: null pointer");
  DVIE_CHECK_ARG(d->ws_k % 4 == 0 || d->ws_k == 1, "wreduce: ws_k=%d", d->ws_k);
  DVIE_CHECK_ARG(((long long)d->co_off * d->ws_k) % 4 == 0 && d->ws_rows * (long long)d->ws_k % 4 == 0,
                 "wreduce: slab alignment (ws_rows*ws_k and co_off*ws_k multiples of 4)");
  DVIE_CHECK_ARG(d->co_off + d->cout_p <= d->ws_rows, "wreduce: rows");
  return DVIE_OK;
}

int dvie_wgrad_reduce_multi(const dvie_wreduce_desc* descs, int n, void* stream) {
  DVIE_CHECK_ARG(descs && n >= 0, "wreduce_multi: args");
  for (int base = 0; base < n; base += WRM) {
    WreduceMulti m;
    m.n = 0;
    int blocks = 0;
    for (int i = base; i < n && i < base + WRM; ++i) {
      const int rc = wreduce_check(&descs[i]);
      if (rc != DVIE_OK) return rc;
      const long long total4 = (long long)(descs[i].ws_rows - descs[i].co_off) * descs[i].ws_k / 4;
      if (total4 < 1) continue;
      m.d[m.n] = descs[i];
      m.blk0[m.n] = blocks;
      blocks += (int)((total4 + 31) / 32);
      ++m.n;
    }
    m.blk0[m.n] = blocks;
    if (m.n == 0) continue;
    DVIE_LAUNCH(wreduce_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, m);
  }
  DVIE_RETURN_LAUNCH();
}

int dvie_colsum(const dvie_colsum_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->g && d->ws && d->c % 4 == 0 && d->c <= 4096, "colsum: args");
  DVIE_CHECK_ARG(d->g_ld % 4 == 0, "colsum: g_ld");
  const long long chunk = (d->rows + d->splits - 1) / d->splits;
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == DVIE_BF16)
    DVIE_LAUNCH(colsum_kernel<bf16_t>, dim3(d->splits), dim3(256), 0, s, *d, chunk);
  else
    DVIE_LAUNCH(colsum_kernel<float>, dim3(d->splits), dim3(256), 0, s, *d, chunk);
  DVIE_RETURN_LAUNCH();
}

int dvie_pack_weights(const dvie_pack_desc* descs_dev, int n, int blocks, void* stream) {
  DVIE_CHECK_ARG(descs_dev && n > 0 && blocks > 0, "pack: args (n %d, blocks %d)", n, blocks);
  DVIE_LAUNCH(pack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, descs_dev, n);
  DVIE_RETURN_LAUNCH();
}

const char* dvie_last_error(void) { return dvie::last_error(); }

int dvie_pack_blocks(const dvie_pack_desc* d) {
  if (!d || d->rows <= 0 || d->kpad <= 0) return 0;
  switch (pack_kind(*d)) {
    case PACK_ROW: return d->rows;
    case PACK_TILE: return cdiv(d->rows, PACK_TR) * cdiv(d->c, PACK_TC);
    default: return cdiv((long long)d->rows * d->kpad, 1024);
  }
}

int dvie_trace_kernels(int on) {
  const int was = dvie::g_trace_on ? 1 : 0;
  dvie::g_trace_on = on != 0;
  dvie::g_trace.clear();
  return was;
}

const char* dvie_traced_kernels(void) {
  dvie::g_trace_text.clear();
  for (size_t i = 0; i < dvie::g_trace.size(); ++i) {
    if (i) dvie::g_trace_text += ';';
    dvie::g_trace_text += dvie::kernel_name(dvie::g_trace[i]);
  }
  dvie::g_trace.clear();
  return dvie::g_trace_text.c_str();
}

}  // extern "C"
