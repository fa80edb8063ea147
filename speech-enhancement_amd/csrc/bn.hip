// Real BatchNorm2d with the activation that follows it fused (CARN / GCARN
// ConvBlock: BatchNorm2d + PReLU, models/_2104_05267_carn.py:30-56; CRN
// ConvBlock: BatchNorm2d + ELU, models/_1809_01405_crn.py:9-45), forward in
// training (batch statistics, running-stat update) and eval mode, and the
// backward. The input may be a row-cropped view (CRN's conv(x)[:, :, :-p, :]):
// every (b, c) plane is HW contiguous floats at x + (b*C + c) * plane_stride.
//
// One workgroup per (b, c) plane for the reductions (fp64 partial sums, no
// atomics), a per-channel finalize that adds the B partials in order, and one
// elementwise apply pass: fwd 2 reads + 1 write of the activation, bwd 2 + 3.
// Storage type T (SE_DTYPE_*): fp32, or bf16 / fp16 for a model.to(bfloat16) /
// .half() module (BASELINE config 5: CARN fp16) -- activations, parameters, running
// statistics and the PReLU weight in T, fp32 / fp64 arithmetic; save stays fp32.
#include "common.hpp"

#include <cmath>

namespace {

constexpr int kThreads = 256;

enum Act { kNone = 0, kPReLU = 1, kELU = 2 };

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = se::wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  __syncthreads();
  return s;
}

struct BnArgs {
  const void* x;
  long long plane;      // x plane stride (elements)
  int B, C, HW;
  const void* weight;   // [C] or null (affine=False)
  const void* bias;
  const void* act_param;    // PReLU weight: [1] or [C]
  int act, act_per_channel;
  float elu_alpha;
};

template <typename T> __device__ __forceinline__ float ldp(const void* p, long long i, float dflt = 0.f) {
  return p ? (float)static_cast<const T*>(p)[i] : dflt;
}
template <typename T> __device__ __forceinline__ void stp(void* p, long long i, float v) {
  static_cast<T*>(p)[i] = (T)v;
}

template <typename T>
__device__ __forceinline__ float act_fwd(const BnArgs& a, int c, float z) {
  if (a.act == kPReLU) {
    const float w = ldp<T>(a.act_param, a.act_per_channel ? c : 0);
    return z >= 0.f ? z : w * z;                         // torch prelu: x > 0 ? x : w x (0 maps to 0 either way)
  }
  if (a.act == kELU) return z > 0.f ? z : a.elu_alpha * (expf(z) - 1.f);
  return z;
}

// d act / dz (as torch's backward formulas: prelu x > 0 ? 1 : w; elu x > 0 ? 1 : y + alpha)
template <typename T>
__device__ __forceinline__ float act_grad(const BnArgs& a, int c, float z) {
  if (a.act == kPReLU) return z > 0.f ? 1.f : ldp<T>(a.act_param, a.act_per_channel ? c : 0);
  if (a.act == kELU) return z > 0.f ? 1.f : a.elu_alpha * expf(z);
  return 1.f;
}

// grid (B, C): sum x, sum x^2 of one plane -> part[(c * B + b) * 2 + {0, 1}]
template <typename T>
__global__ void __launch_bounds__(kThreads) bn_moments_kernel(BnArgs a, double* __restrict__ part) {
  const int b = blockIdx.x, c = blockIdx.y;
  const T* x = static_cast<const T*>(a.x) + ((long long)b * a.C + c) * a.plane;
  __shared__ double red[kThreads / 64];
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < a.HW; i += kThreads) {
    const double v = (float)x[i];
    s += v;
    ss += v * v;
  }
  s = block_sum(s, red);
  ss = block_sum(ss, red);
  if (threadIdx.x == 0) {
    part[((long long)c * a.B + b) * 2] = s;
    part[((long long)c * a.B + b) * 2 + 1] = ss;
  }
}

// one thread per channel: mean, biased var -> save = {mean, invstd}; running
// stats as torch: r = (1 - m) r + m * stat (running_var with the unbiased var)
template <typename T>
__global__ void bn_finalize_kernel(const double* __restrict__ part, int B, int C, long long n, float eps,
                                   float momentum, void* __restrict__ rmean, void* __restrict__ rvar,
                                   float* __restrict__ save) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0, ss = 0;
  for (int b = 0; b < B; ++b) {
    s += part[((long long)c * B + b) * 2];
    ss += part[((long long)c * B + b) * 2 + 1];
  }
  const double mean = s / n;
  const double var = fmax(ss / n - mean * mean, 0.0);
  save[c] = (float)mean;
  save[C + c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    stp<T>(rmean, c, (1.f - momentum) * ldp<T>(rmean, c) + momentum * (float)mean);
    const double unbiased = n > 1 ? var * n / (n - 1) : var;
    stp<T>(rvar, c, (1.f - momentum) * ldp<T>(rvar, c) + momentum * (float)unbiased);
  }
}

// eval: save = {running mean, 1 / sqrt(running var + eps)}
template <typename T>
__global__ void bn_eval_stats_kernel(const void* __restrict__ rmean, const void* __restrict__ rvar, int C,
                                     float eps, float* __restrict__ save) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  save[c] = ldp<T>(rmean, c);
  save[C + c] = 1.f / sqrtf(ldp<T>(rvar, c) + eps);
}

// grid (ceil(HW / (4 kThreads)), B * C): y = act((x - mean) * invstd * w + b)
template <typename T>
__global__ void __launch_bounds__(kThreads)
bn_apply_kernel(BnArgs a, const float* __restrict__ save, T* __restrict__ y) {
  const int bc = blockIdx.y, c = bc % a.C;
  const float mean = save[c], inv = save[a.C + c];
  const float w = ldp<T>(a.weight, c, 1.f), bb = ldp<T>(a.bias, c, 0.f);
  const T* x = static_cast<const T*>(a.x) + (long long)bc * a.plane;
  T* yo = y + (long long)bc * a.HW;
  for (int u = 0; u < 4; ++u) {
    const int i = (blockIdx.x * 4 + u) * kThreads + threadIdx.x;
    if (i >= a.HW) return;
    yo[i] = (T)act_fwd<T>(a, c, ((float)x[i] - mean) * inv * w + bb);
  }
}

// grid (B, C): per plane sum g, sum g * xhat, and the PReLU weight partial
// sum gy * z [z <= 0] (g = gy * act'(z), z recomputed from x)
template <typename T>
__global__ void __launch_bounds__(kThreads)
bn_bwd_moments_kernel(BnArgs a, const T* __restrict__ gy, const float* __restrict__ save,
                      double* __restrict__ part) {
  const int b = blockIdx.x, c = blockIdx.y;
  const float mean = save[c], inv = save[a.C + c];
  const float w = ldp<T>(a.weight, c, 1.f), bb = ldp<T>(a.bias, c, 0.f);
  const T* x = static_cast<const T*>(a.x) + ((long long)b * a.C + c) * a.plane;
  const T* g = gy + ((long long)b * a.C + c) * a.HW;
  __shared__ double red[kThreads / 64];
  double sg = 0, sgx = 0, sa = 0;
  for (int i = threadIdx.x; i < a.HW; i += kThreads) {
    const float xh = ((float)x[i] - mean) * inv;
    const float z = xh * w + bb;
    const float gi = (float)g[i];
    const float gz = gi * act_grad<T>(a, c, z);
    sg += gz;
    sgx += (double)gz * xh;
    if (a.act == kPReLU && !(z > 0.f)) sa += (double)gi * z;
  }
  sg = block_sum(sg, red);
  sgx = block_sum(sgx, red);
  if (a.act == kPReLU) sa = block_sum(sa, red);
  if (threadIdx.x == 0) {
    double* p = part + ((long long)c * a.B + b) * 3;
    p[0] = sg; p[1] = sgx; p[2] = sa;
  }
}

// one thread per channel: dbias = sum g, dweight = sum g xhat, and the
// per-channel means the dx pass needs -> red[c] = {sum g / n, sum g xhat / n};
// PReLU: per-channel weight grads, or (shared weight) channel partials summed
// by bn_act_param_kernel
template <typename T>
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ part, int B, int C, long long n, int act,
                                       int act_per_channel, void* __restrict__ dweight, void* __restrict__ dbias,
                                       void* __restrict__ dact, double* __restrict__ act_part,
                                       float* __restrict__ red) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg = 0, sgx = 0, sa = 0;
  for (int b = 0; b < B; ++b) {
    const double* p = part + ((long long)c * B + b) * 3;
    sg += p[0];
    sgx += p[1];
    sa += p[2];
  }
  if (dweight) stp<T>(dweight, c, (float)sgx);
  if (dbias) stp<T>(dbias, c, (float)sg);
  red[c] = (float)(sg / n);
  red[C + c] = (float)(sgx / n);
  if (act == kPReLU) {
    if (act_per_channel) stp<T>(dact, c, (float)sa);
    else act_part[c] = sa;
  }
}

template <typename T>
__global__ void bn_act_param_kernel(const double* __restrict__ act_part, int C, void* __restrict__ dact) {
  __shared__ double r[kThreads / 64];
  double s = 0;
  for (int c = threadIdx.x; c < C; c += kThreads) s += act_part[c];
  s = block_sum(s, r);
  if (threadIdx.x == 0) stp<T>(dact, 0, (float)s);
}

// grid (ceil(HW / (4 kThreads)), B * C): train dx = w inv (g - mean g - xhat mean(g xhat)); eval dx = w inv g
template <typename T>
__global__ void __launch_bounds__(kThreads)
bn_bwd_apply_kernel(BnArgs a, const T* __restrict__ gy, const float* __restrict__ save,
                    const float* __restrict__ red, int training, T* __restrict__ dx) {
  const int bc = blockIdx.y, c = bc % a.C;
  const float mean = save[c], inv = save[a.C + c];
  const float w = ldp<T>(a.weight, c, 1.f), bb = ldp<T>(a.bias, c, 0.f);
  const float mg = training ? red[c] : 0.f, mgx = training ? red[a.C + c] : 0.f;
  const T* x = static_cast<const T*>(a.x) + (long long)bc * a.plane;
  const T* g = gy + (long long)bc * a.HW;
  T* d = dx + (long long)bc * a.HW;
  for (int u = 0; u < 4; ++u) {
    const int i = (blockIdx.x * 4 + u) * kThreads + threadIdx.x;
    if (i >= a.HW) return;
    const float xh = ((float)x[i] - mean) * inv;
    const float gz = (float)g[i] * act_grad<T>(a, c, xh * w + bb);
    d[i] = (T)(w * inv * (gz - mg - xh * mgx));
  }
}

int check(const BnArgs& a) {
  if (!a.x || a.B <= 0 || a.C <= 0 || a.HW <= 0 || a.plane < a.HW) return SE_E_ARG;
  if (a.act < kNone || a.act > kELU || (a.act == kPReLU && !a.act_param)) return SE_E_ARG;
  return SE_OK;
}

}  // namespace

extern "C" size_t se_bn_workspace_size(int B, int C) {
  return (B > 0 && C > 0) ? (size_t)B * C * 3 * sizeof(double) + (size_t)C * (sizeof(double) + 2 * sizeof(float)) + 512
                          : 0;
}

namespace {

template <typename T>
int bn_fwd_t(const BnArgs& a, void* running_mean, void* running_var, int training, float momentum, float eps, T* y,
             float* save, void* ws, hipStream_t st) {
  const int B = a.B, C = a.C, HW = a.HW;
  if (training) {
    double* part = (double*)ws;
    hipLaunchKernelGGL(bn_moments_kernel<T>, dim3(B, C), dim3(kThreads), 0, st, a, part);
    SE_LAUNCH_CHECK();
    hipLaunchKernelGGL(bn_finalize_kernel<T>, dim3(se::ceil_div(C, 64)), dim3(64), 0, st, part, B, C,
                       (long long)B * HW, eps, momentum, running_mean, running_var, save);
  } else {
    hipLaunchKernelGGL(bn_eval_stats_kernel<T>, dim3(se::ceil_div(C, 64)), dim3(64), 0, st,
                       (const void*)running_mean, (const void*)running_var, C, eps, save);
  }
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(se::ceil_div(HW, 4 * kThreads), B * C), dim3(kThreads), 0, st, a,
                     (const float*)save, y);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

template <typename T>
int bn_bwd_t(const BnArgs& a, const T* gy, const float* save, int training, T* dx, void* dweight, void* dbias,
             void* dact_param, void* ws, hipStream_t st) {
  const int B = a.B, C = a.C, HW = a.HW;
  double* part = (double*)ws;
  double* act_part = part + (size_t)B * C * 3;
  float* red = (float*)(act_part + C);
  hipLaunchKernelGGL(bn_bwd_moments_kernel<T>, dim3(B, C), dim3(kThreads), 0, st, a, gy, save, part);
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<T>, dim3(se::ceil_div(C, 64)), dim3(64), 0, st, (const double*)part, B,
                     C, (long long)B * HW, a.act, a.act_per_channel, dweight, dbias, dact_param, act_part, red);
  SE_LAUNCH_CHECK();
  if (a.act == kPReLU && !a.act_per_channel) {
    hipLaunchKernelGGL(bn_act_param_kernel<T>, dim3(1), dim3(kThreads), 0, st, (const double*)act_part, C,
                       dact_param);
    SE_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(se::ceil_div(HW, 4 * kThreads), B * C), dim3(kThreads), 0, st,
                     a, gy, save, (const float*)red, training, dx);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

}  // namespace

extern "C" int se_bn_fwd(const void* x, long long x_plane_stride, int B, int C, int HW, const void* weight,
                         const void* bias, void* running_mean, void* running_var, int training, float momentum,
                         float eps, int act, const void* act_param, int act_per_channel, float elu_alpha, void* y,
                         float* save, int dtype, void* ws, size_t ws_bytes, void* stream) {
  BnArgs a{x, x_plane_stride, B, C, HW, weight, bias, act_param, act, act_per_channel, elu_alpha};
  int rc = check(a);
  if (rc) return rc;
  if (!y || !save || (!training && (!running_mean || !running_var)) || (!running_mean != !running_var))
    return SE_E_ARG;
  if (training && (!ws || ws_bytes < se_bn_workspace_size(B, C))) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  switch (dtype) {
    case SE_DTYPE_F32:
      return bn_fwd_t<float>(a, running_mean, running_var, training, momentum, eps, (float*)y, save, ws, st);
    case SE_DTYPE_BF16:
      return bn_fwd_t<__bf16>(a, running_mean, running_var, training, momentum, eps, (__bf16*)y, save, ws, st);
    case SE_DTYPE_F16:
      return bn_fwd_t<_Float16>(a, running_mean, running_var, training, momentum, eps, (_Float16*)y, save, ws, st);
    default:
      return SE_E_ARG;
  }
}

extern "C" int se_bn_bwd(const void* gy, const void* x, long long x_plane_stride, int B, int C, int HW,
                         const void* weight, const void* bias, const float* save, int training, int act,
                         const void* act_param, int act_per_channel, float elu_alpha, void* dx, void* dweight,
                         void* dbias, void* dact_param, int dtype, void* ws, size_t ws_bytes, void* stream) {
  BnArgs a{x, x_plane_stride, B, C, HW, weight, bias, act_param, act, act_per_channel, elu_alpha};
  int rc = check(a);
  if (rc) return rc;
  if (!gy || !save || !dx || (act == kPReLU && !dact_param)) return SE_E_ARG;
  if (!ws || ws_bytes < se_bn_workspace_size(B, C)) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  switch (dtype) {
    case SE_DTYPE_F32:
      return bn_bwd_t<float>(a, (const float*)gy, save, training, (float*)dx, dweight, dbias, dact_param, ws, st);
    case SE_DTYPE_BF16:
      return bn_bwd_t<__bf16>(a, (const __bf16*)gy, save, training, (__bf16*)dx, dweight, dbias, dact_param, ws, st);
    case SE_DTYPE_F16:
      return bn_bwd_t<_Float16>(a, (const _Float16*)gy, save, training, (_Float16*)dx, dweight, dbias, dact_param,
                                ws, st);
    default:
      return SE_E_ARG;
  }
}
