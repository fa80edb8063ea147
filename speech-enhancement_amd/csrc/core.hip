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
