// ABI housekeeping: version, error strings, loader self-test kernel.
#include "common.hpp"

extern "C" int se_abi_version(void) { return SEHIP_ABI_VERSION; }

extern "C" const char* se_strerror(int code) {
  switch (code) {
    case SE_OK: return "ok";
    case SE_E_ARG: return "invalid argument";
    case SE_E_SHAPE: return "inconsistent shape";
    case SE_E_UNSUPPORTED: return "unsupported configuration";
    case SE_E_LAUNCH: return "kernel launch failed";
    case SE_E_WORKSPACE: return "workspace too small";
    default: return "unknown sehip error";
  }
}

__global__ void probe_kernel(int* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = 3 * i + 1;
}

extern "C" int se_probe(int* out, int n, void* stream) {
  if (!out || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  hipLaunchKernelGGL(probe_kernel, dim3(se::ceil_div(n, 256)), dim3(256), 0,
                     se::as_stream(stream), out, n);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

// A HIP stream restricted to a subset of the CUs (hipExtStreamCreateWithCUMask):
// CU i is enabled when (i % den) < num. Used for the deferred weight-grad side
// stream, so the MFMA-bound weight-grads cannot take the CUs the main stream's
// HBM-bound passes need.
extern "C" int se_stream_create_cu_subset(int num, int den, void** stream) {
  if (!stream || den <= 0 || num <= 0 || num > den) return SE_E_ARG;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SE_E_LAUNCH;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return SE_E_LAUNCH;
  const int words = (cus + 31) / 32;
  uint32_t mask[64] = {0};
  if (words > 64) return SE_E_UNSUPPORTED;
  for (int i = 0; i < cus; ++i)
    if ((i % den) < num) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return SE_E_LAUNCH;
  *stream = (void*)s;
  return SE_OK;
}

extern "C" int se_stream_destroy(void* stream) {
  if (!stream) return SE_E_ARG;
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? SE_OK : SE_E_LAUNCH;
}
