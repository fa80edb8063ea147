// Shared helpers for the sehip HIP kernels (gfx950 / CDNA4 only).
//
// Conventions (see include/sehip.h):
//   * every entry point returns 0 on success or a negative SE_E* code;
//   * every launch goes onto the caller's hipStream_t, nothing synchronises;
//   * the library allocates nothing: scratch comes in as a workspace pointer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/sehip.h"

#define SE_LAUNCH_CHECK()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return SE_E_LAUNCH;               \
  } while (0)

namespace se {

constexpr int kWave = 64;

// A 64-bit pointer from its two 32-bit words. Both words are unsigned: widening a
// signed low word (what __builtin_amdgcn_readfirstlane returns) sign-extends any
// address whose low word is >= 2^31 into the high word (the d630867 fault in the
// chunked stencil). tests/test_uniform_ptr_cpu.py checks this on the host.
__host__ __device__ __forceinline__ unsigned long long ptr_from_words(unsigned lo, unsigned hi) {
  return ((unsigned long long)hi << 32) | lo;
}

// p made provably wave-uniform (readfirstlane on both halves) for a buffer resource
// base; otherwise hipcc wraps every buffer op in a waterfall loop.
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const unsigned long long v = (unsigned long long)p;
  return (void*)ptr_from_words((unsigned)__builtin_amdgcn_readfirstlane((unsigned)v),
                               (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// SE_MATH_F16X3 operand scaling (the conv and LSTM GEMMs): a tensor with max |x| <= *amax < 2^e is
// multiplied by s = 2^(kF16Top - e), so every scaled value is below 2^14 (fp16 max
// 65504), then split as hi = fp16(x s), lo = fp16(x s - hi) (x s - hi is exact).
constexpr int kF16Top = 14;
// e with *amax < 2^e (from the fp32 exponent field; 0 and denormals -> -126),
// clamped so that 2^(kF16Top - e) is a normal float
__device__ __forceinline__ int amax_exp(const float* amax) {
  const unsigned bits = __builtin_bit_cast(unsigned, *amax) & 0x7fffffffu;
  const int e = (int)(bits >> 23) - 126;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}
__device__ __forceinline__ float pow2f(int e) { return __builtin_bit_cast(float, (unsigned)(127 + e) << 23); }
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
// (x0, x1) * s -> packed fp16 hi pair and lo pair (element 0 in the low half);
// v_cvt_pk_f16_f32 rounds to nearest even
__device__ __forceinline__ void split_f16x2(float x0, float x1, float s, unsigned& hi, unsigned& lo) {
  const f32x2v v = (f32x2v){x0, x1} * s;
  const f16x2v h = __builtin_convertvector(v, f16x2v);
  hi = __builtin_bit_cast(unsigned, h);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(v - __builtin_convertvector(h, f32x2v), f16x2v));
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace se
