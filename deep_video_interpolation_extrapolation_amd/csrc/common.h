// Shared device helpers for the gfx950 kernels (bf16 <-> f32, 4-channel vectors,
// activation functions and their output-side derivatives, error plumbing).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/dvie.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

typedef uint16_t bf16_t;  // raw bf16 storage

namespace dvie {

void set_error(const char* fmt, ...);

#define DVIE_CHECK_ARG(cond, ...)      \
  do {                                 \
    if (!(cond)) {                     \
      ::dvie::set_error(__VA_ARGS__);  \
      return DVIE_EINVAL;              \
    }                                  \
  } while (0)

// Timing-only ablation switches (DVIE_1X1_DBG / DVIE_HALO_DBG / DVIE_NARROW_DBG / DVIE_SEGENC_DBG skip stores,
// MFMAs or operand streams, so results are wrong) exist only in a build made with
// -DDVIE_TIMING_DBG; in the product build the kernels see a constant 0 and the host never
// reads those variables.
#ifdef DVIE_TIMING_DBG
#define DVIE_DBG(x) (x)
#else
#define DVIE_DBG(x) 0
#endif

// Launch trace (diagnostics: dvie_trace_kernels / dvie_traced_kernels in include/dvie.h).
// Every kernel launch of the library goes through DVIE_LAUNCH, which notes the kernel's host
// stub when the calling thread has tracing on (one thread-local flag test otherwise).
extern thread_local bool g_trace_on;
void trace_launch(const void* fn);
#define DVIE_LAUNCH(kern, ...)                                                       \
  do {                                                                               \
    if (::dvie::g_trace_on) ::dvie::trace_launch(reinterpret_cast<const void*>(kern)); \
    hipLaunchKernelGGL(kern, __VA_ARGS__);                                           \
  } while (0)

#define DVIE_RETURN_LAUNCH()                     \
  do {                                           \
    hipError_t _e = hipGetLastError();           \
    return _e == hipSuccess ? DVIE_OK : (int)_e; \
  } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN kept NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// 4-element vector access (fp32: 16 B, bf16: 8 B)
template <typename T>
struct V4;
template <>
struct V4<float> {
  __device__ __forceinline__ static f32x4 load(const float* p) { return *(const f32x4*)p; }
  __device__ __forceinline__ static void store(float* p, f32x4 v) { *(f32x4*)p = v; }
};
template <>
struct V4<bf16_t> {
  __device__ __forceinline__ static f32x4 load(const bf16_t* p) {
    i32x2 r = *(const i32x2*)p;
    f32x4 v;
    v[0] = __uint_as_float(((uint32_t)r[0]) << 16);
    v[1] = __uint_as_float(((uint32_t)r[0]) & 0xffff0000u);
    v[2] = __uint_as_float(((uint32_t)r[1]) << 16);
    v[3] = __uint_as_float(((uint32_t)r[1]) & 0xffff0000u);
    return v;
  }
  __device__ __forceinline__ static void store(bf16_t* p, f32x4 v) {
    i32x2 r;
    r[0] = (int)((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16));
    r[1] = (int)((uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    *(i32x2*)p = r;
  }
};

__device__ __forceinline__ float act_fwd(float v, int act, float alpha) {
  switch (act) {
    case DVIE_ACT_LRELU: return v > 0.f ? v : v * alpha;
    case DVIE_ACT_ELU: return v > 0.f ? v : expm1f(v);
    case DVIE_ACT_RELU: return v > 0.f ? v : 0.f;
    case DVIE_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// ELU / tanh for the bf16-output kernels: v_exp_f32-based forms, a few instructions each
// instead of the libm expansions (which, inlined for every output element of an unrolled
// epilogue, made those kernels 10-14K instructions long).  Accuracy: expm1 within ~2e-7
// absolute (Taylor below |v| = 1/32), tanh within ~2e-7 absolute (odd Taylor below 1/64) --
// far inside the bf16 rounding of the stored result.
__device__ __forceinline__ float elu_bf(float v) {
  const float t = v > -0.03125f ? v * (1.f + v * (0.5f + v * (1.f / 6.f))) : __expf(v) - 1.f;
  return v > 0.f ? v : t;
}
__device__ __forceinline__ float tanh_bf(float v) {
  const float a = fabsf(v), e = __expf(-2.f * a);
  const float t = a < 0.015625f ? a * (1.f - a * a * (1.f / 3.f)) : (1.f - e) * __frcp_rn(1.f + e);
  return copysignf(t, v);
}
__device__ __forceinline__ float act_bf(float v, int act, float alpha) {
  switch (act) {
    case DVIE_ACT_LRELU: return v > 0.f ? v : v * alpha;
    case DVIE_ACT_ELU: return elu_bf(v);
    case DVIE_ACT_RELU: return v > 0.f ? v : 0.f;
    case DVIE_ACT_TANH: return tanh_bf(v);
    default: return v;
  }
}

// the same activations for fp32-output epilogues (fp32 head outputs of a bf16 plan): libm
// expm1f / tanhf, not the short forms above, which are accurate to bf16 rounding only
__device__ __forceinline__ float act_f32(float v, int act, float alpha) {
  switch (act) {
    case DVIE_ACT_LRELU: return v > 0.f ? v : v * alpha;
    case DVIE_ACT_ELU: return v > 0.f ? v : expm1f(v);
    case DVIE_ACT_RELU: return v > 0.f ? v : 0.f;
    case DVIE_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// derivative expressed through the activation OUTPUT z
__device__ __forceinline__ float act_dz(float z, int act, float alpha) {
  switch (act) {
    case DVIE_ACT_LRELU: return z > 0.f ? 1.f : alpha;
    case DVIE_ACT_ELU: return z > 0.f ? 1.f : z + 1.f;
    case DVIE_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case DVIE_ACT_TANH: return 1.f - z * z;
    default: return 1.f;
  }
}

__host__ __device__ __forceinline__ int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// One LDS-DMA piece (buffer_load_dwordx4 ... lds: 64 lanes x 16 B into LDS at dst + 16 * lane)
// issued through inline asm.  With __builtin_amdgcn_raw_ptr_buffer_load_lds the compiler
// sees an LDS write behind the load and puts s_waitcnt vmcnt(0) before the next LDS read, so
// a next-tile prefetch issued before the current tile's MFMAs is waited for before those
// MFMAs start (no overlap at all).  Kernels that use this order LDS themselves: counted
// s_waitcnt vmcnt + barrier before reading what the DMA wrote.  (s_nop 0: the one wait state
// an SALU write of M0 needs before an LDS-DMA reads it.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, const void* dst, unsigned voff) {
  typedef __attribute__((address_space(3))) void* lds_vp;
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_vp)(void*)dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r) : "memory", "m0");
}
#pragma clang diagnostic pop

}  // namespace dvie
