// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors travel as raw `uint16_t` bit patterns; math is fp32.
//   * wave = 64 lanes (hard-coded, never warpSize-32 idioms).
//   * global loads of bf16 are 16-byte vectors (8 elements) wherever the
//     shape allows (MI355X guide, Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Device debug flavour (csrc/build.py --debug defines SHAI_KERNEL_DEBUG): SHAI_DASSERT bounds-checks DMA offsets,
// LDS indices and ring slot ids in the hand-scheduled kernels (a failing check prints its condition and aborts the
// kernel), and SHAI_DEBUG selects hazard-safe forms of hand-counted waits (vmcnt(0) for counted vmcnt(N), wider
// s_nop margins after inline-asm MFMAs).  Both compile to nothing in the production build.
#ifdef SHAI_KERNEL_DEBUG
#include <cassert>
#define SHAI_DASSERT(c) assert(c)
#define SHAI_DEBUG 1
#else
#define SHAI_DASSERT(c) ((void)0)
#define SHAI_DEBUG 0
#endif

namespace shai {

constexpr int kWave = 64;

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4 __attribute__((ext_vector_type(4)));
typedef float float4_ __attribute__((ext_vector_type(4)));
typedef float float16_ __attribute__((ext_vector_type(16)));
typedef uint32_t uint4_ __attribute__((ext_vector_type(4)));
typedef uint32_t uint2_ __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t x) { return __uint_as_float(x << 16); }

// Round-to-nearest-even fp32 -> bf16 (plain cast lowers to v_cvt_pk_bf16_f32
// on gfx950 and keeps NaNs NaN).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// Unpack 8 bf16 held in a uint4 into fp32.
__device__ __forceinline__ void unpack8(const uint4_ v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4_ pack8(const float* f) {
  uint4_ v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack2(f[2 * i], f[2 * i + 1]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Activations divide with v_rcp_f32 (1 ulp): a plain '/' or __frcp_rn expands to the correctly rounded
// v_div_scale / v_div_fmas / v_div_fixup sequence (~10 instructions), which made the GEGLU epilogue of the
// W-stationary GEMM VALU-bound (120 such sequences per tile step).
__device__ __forceinline__ float rcp_f(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float silu_f(float x) { return x * rcp_f(1.0f + __expf(-x)); }

// erf via Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16 resolution): one exp, one
// reciprocal and a degree-5 Horner chain instead of the libm erff polynomial + branches, which
// made GEGLU epilogues VALU-bound.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = rcp_f(fmaf(0.3275911f, ax, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y = 1.0f - y * t * __expf(-ax * ax);
  return copysignf(y, x);
}

// gelu(x) = x/2 + |x|/2 * erf(|x| / sqrt 2), the same 7.1.26 erf written for the GELU argument directly: the
// 1/sqrt 2 and log2 e factors folded into the constants, the sign handled by the |x|/2 form (no copysign):
// 13 VALU, 2 of them transcendental.
__device__ __forceinline__ float gelu_erf_f(float x) {
  const float hx = 0.5f * x;
  const float t = rcp_f(fmaf(0.23164189f, fabsf(x), 1.0f));  // 0.3275911 / sqrt 2
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752f);  // exp(-x^2 / 2)
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  const float erf_abs = fmaf(-(y * t), e, 1.0f);
  return fmaf(fabsf(hx), erf_abs, hx);
}

// tanh(u) = 1 - 2 / (1 + e^{2u}) (saturates correctly at +-1 for large |u|)
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * fmaf(k1 * x, x * x, x);
  const float th = 1.0f - 2.0f * rcp_f(1.0f + __expf(2.0f * u));
  return 0.5f * x * (1.0f + th);
}

__device__ __forceinline__ float quick_gelu_f(float x) { return x * rcp_f(1.0f + __expf(-1.702f * x)); }

// smallest bf16-representable float >= x (finite x; -inf stays -inf): flash attention keeps its running max on
// the bf16 grid so that -m can enter the score MFMA exactly as a bf16 operand
__device__ __forceinline__ float bf16_up(float x) {
  uint32_t u = __float_as_uint(x);
  if ((u & 0xffffu) == 0u) return x;
  if (!(u >> 31)) u += 0x10000u;  // positive: round the magnitude up; negative: truncation rounds up
  return __uint_as_float(u & 0xffff0000u);
}

enum Act : int { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_GELU_TANH = 3, ACT_QUICK_GELU = 4, ACT_RELU = 5 };

template <int ACT>
__device__ __forceinline__ float apply_act(float x) {
  if constexpr (ACT == ACT_SILU) return silu_f(x);
  else if constexpr (ACT == ACT_GELU) return gelu_erf_f(x);
  else if constexpr (ACT == ACT_GELU_TANH) return gelu_tanh_f(x);
  else if constexpr (ACT == ACT_QUICK_GELU) return quick_gelu_f(x);
  else if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  else return x;
}

__device__ __forceinline__ float apply_act_rt(int act, float x) {
  switch (act) {
    case ACT_SILU: return silu_f(x);
    case ACT_GELU: return gelu_erf_f(x);
    case ACT_GELU_TANH: return gelu_tanh_f(x);
    case ACT_QUICK_GELU: return quick_gelu_f(x);
    case ACT_RELU: return fmaxf(x, 0.f);
    default: return x;
  }
}

}  // namespace shai

#define SHAI_CHECK_LAUNCH() (void)hipGetLastError()

// debug check of a 16-B buffer-DMA offset against its buffer: in range, or the out-of-bounds zero-fill sentinel
// (any offset at or above the sentinel is out of the <= 2^31-byte buffer range: zero fill)
#define SHAI_DASSERT_DMA(off, bytes, oob) \
  SHAI_DASSERT((uint32_t)(off) >= (uint32_t)(oob) || (long)(off) + 16 <= (long)(bytes))
