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

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace se
