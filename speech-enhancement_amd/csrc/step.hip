// Train-step glue: the loss and the parameter update of
// one iteration of the reference's hot loop, as a handful of launches instead
// of dozens of ATen reductions and foreach kernels.
//
//  * SI-SNR (losses.py:62-84) with utils.py:111-121's pad / truncate of the
//    estimate folded into the reads: one workgroup per utterance (fp64 sums),
//    one finalize launch for the batch mean; the backward is one elementwise
//    pass from the saved per-utterance sums.
//  * clip_grad_norm_(max_norm) + AdamW.step (trainer.py:216-221) over a device
//    table of parameter slots (the virtual concatenation of every tensor):
//    one sum-of-squares launch, one clip launch, one AdamW launch per step.
#include "common.hpp"

#include <cmath>

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 8192;     // elements per workgroup iteration of the slot kernels

template <typename T, int NT = kThreads>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = se::wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) s += red[w];
  __syncthreads();
  return s;
}

constexpr int kItemThreads = 1024;   // one workgroup per utterance: the whole CU

// per-utterance save: [0] mean e, [1] mean t, [2] dot (fp32), [3] |t|^2 (fp32),
// [4] S, [5] N, [6] sum p, [7] sum (e' - p)  (doubles)
constexpr int kSave = 8;

template <typename T>
__device__ __forceinline__ float rt(float v) { return (float)(T)v; }

template <typename T>
__global__ void __launch_bounds__(kItemThreads)
sisnr_items_kernel(const T* __restrict__ est, int le, long long est_stride, const T* __restrict__ tgt, int lt,
                   int zero_mean, double* __restrict__ save) {
  const int b = blockIdx.x;
  const T* e = est + (long long)b * est_stride;
  const T* t = tgt + (long long)b * lt;
  const int ne = min(le, lt);                 // estimate samples inside the target length
  __shared__ double red[kItemThreads / 64];
  float me = 0.f, mt = 0.f;
  if (zero_mean) {
    double se_ = 0, st = 0;
    for (int i = threadIdx.x; i < lt; i += kItemThreads) {
      se_ += i < ne ? (float)e[i] : 0.f;
      st += (float)t[i];
    }
    me = (float)(block_sum<double, kItemThreads>(se_, red) / lt);
    mt = (float)(block_sum<double, kItemThreads>(st, red) / lt);
  }
  double dot = 0, tt = 0;
  for (int i = threadIdx.x; i < lt; i += kItemThreads) {
    const float ei = (i < ne ? (float)e[i] : 0.f) - me, ti = (float)t[i] - mt;
    dot += (double)ei * ti;
    tt += (double)ti * ti;
  }
  const float dotf = (float)block_sum<double, kItemThreads>(dot, red), ttf = (float)block_sum<double, kItemThreads>(tt, red);
  double S = 0, Nn = 0, sp = 0, sr = 0;
  for (int i = threadIdx.x; i < lt; i += kItemThreads) {
    const float ei = (i < ne ? (float)e[i] : 0.f) - me, ti = (float)t[i] - mt;
    const float p = dotf * ti / ttf;          // proj = sum(e*t) * t / t_energy
    const float r = ei - p;
    S += (double)p * p;
    Nn += (double)r * r;
    sp += p;
    sr += r;
  }
  S = block_sum<double, kItemThreads>(S, red);
  Nn = block_sum<double, kItemThreads>(Nn, red);
  sp = block_sum<double, kItemThreads>(sp, red);
  sr = block_sum<double, kItemThreads>(sr, red);
  if (threadIdx.x == 0) {
    double* s = save + (long long)b * kSave;
    s[0] = me; s[1] = mt; s[2] = dotf; s[3] = ttf; s[4] = S; s[5] = Nn; s[6] = sp; s[7] = sr;
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
sisnr_finalize_kernel(const double* __restrict__ save, int B, float eps, T* __restrict__ loss) {
  __shared__ double red[kThreads / 64];
  double acc = 0;
  for (int b = threadIdx.x; b < B; b += kThreads) {
    const double* s = save + (long long)b * kSave;
    const float sig = (float)s[4] + eps, noi = (float)s[5] + eps;
    acc += (double)(10.f * log10f(sig / noi));
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) loss[0] = (T)(float)(-acc / B);
}

// grid (ceil(le / kThreads / 4), B): d est[b, i] for i < le (0 past the target length)
template <typename T>
__global__ void __launch_bounds__(kThreads)
sisnr_bwd_kernel(const T* __restrict__ est, int le, long long est_stride, const T* __restrict__ tgt, int lt,
                 int B, int zero_mean, float eps, const double* __restrict__ save, const T* __restrict__ gloss,
                 T* __restrict__ gest, long long g_stride) {
  const int b = blockIdx.y;
  const double* s = save + (long long)b * kSave;
  const float me = (float)s[0], mt = (float)s[1], dotf = (float)s[2], ttf = (float)s[3];
  const float sig = (float)s[4] + eps, noi = (float)s[5] + eps;
  // L_b = 10 log10(sig / noi); loss = -mean_b L_b
  const float k = -(float)gloss[0] * 10.f / ((float)B * 2.302585093f);
  const float cs = 2.f * k / sig, cn = -2.f * k / noi;      // dL/dp-part, dL/d(e'-p)-part
  const float gmean = zero_mean ? (float)((cs * s[6] + cn * s[7]) / lt) : 0.f;
  const T* e = est + (long long)b * est_stride;
  const T* t = tgt + (long long)b * lt;
  const int ne = min(le, lt);
  for (int u = 0; u < 4; ++u) {
    const int i = (blockIdx.x * 4 + u) * kThreads + threadIdx.x;
    if (i >= le) return;
    float g = 0.f;
    if (i < ne) {
      const float ei = (float)e[i] - me, ti = (float)t[i] - mt;
      const float p = dotf * ti / ttf;
      g = cs * p + cn * (ei - p) - gmean;
    }
    gest[(long long)b * g_stride + i] = (T)g;
  }
}

// ------------------------------------------------------------------ slots
struct Slot {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long numel;
  long long offset;   // prefix sum of numel (slots in offset order)
};
static_assert(sizeof(Slot) == sizeof(se_tensor_slot), "Slot mirrors se_tensor_slot");

__device__ __forceinline__ int find_slot(const Slot* slots, int n, long long pos) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (slots[mid].offset <= pos) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Visit every element of the concatenation: f(slot, index in slot).
template <typename F>
__device__ __forceinline__ void for_each_elem(const Slot* slots, int nslots, long long total, F f) {
  for (long long c0 = (long long)blockIdx.x * kChunk; c0 < total; c0 += (long long)gridDim.x * kChunk) {
    const long long c1 = min(total, c0 + kChunk);
    int s = find_slot(slots, nslots, c0);
    long long pos = c0;
    while (pos < c1) {
      const Slot sl = slots[s];
      const long long end = min(c1, sl.offset + sl.numel);
      for (long long i = pos + threadIdx.x; i < end; i += kThreads) f(sl, i - sl.offset);
      pos = end;
      ++s;
    }
  }
}

// per-workgroup partial sums into out[1 + blockIdx.x]; sumsq_final_kernel adds
// them in a fixed order into out[0] (deterministic, unlike fp64 atomics)
template <typename T>
__global__ void __launch_bounds__(kThreads)
sumsq_kernel(const Slot* __restrict__ slots, int nslots, long long total, double* __restrict__ out) {
  __shared__ double red[kThreads / 64];
  double acc = 0;
  for_each_elem(slots, nslots, total, [&](const Slot& s, long long i) {
    const float g = (float)reinterpret_cast<const T*>(s.grad)[i];
    acc += (double)g * g;
  });
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[1 + blockIdx.x] = acc;
}

__global__ void __launch_bounds__(kThreads)
sumsq_final_kernel(double* __restrict__ out, int nparts) {
  __shared__ double red[kThreads / 64];
  double acc = 0;
  for (int i = threadIdx.x; i < nparts; i += kThreads) acc += out[1 + i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = acc;
}

// torch.nn.utils.clip_grad_norm_: coef = max_norm / (total_norm + 1e-6),
// clamped to 1, every gradient multiplied by it. 16-bit gradients: torch's norms are
// tensors of the gradients' dtype, so the total norm, its + 1e-6, the coefficient and
// every product are rounded to it
template <typename T>
__global__ void __launch_bounds__(kThreads)
clip_kernel(const Slot* __restrict__ slots, int nslots, long long total, const double* __restrict__ sumsq,
            float max_norm, float* __restrict__ norm_out) {
  const float tn = rt<T>((float)sqrt(*sumsq));
  const float coef = fminf(rt<T>(max_norm / rt<T>(tn + 1e-6f)), 1.f);
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = tn;
  for_each_elem(slots, nslots, total, [&](const Slot& s, long long i) {
    T* g = reinterpret_cast<T*>(s.grad);
    g[i] = (T)((float)g[i] * coef);
  });
}

// torch.optim.AdamW (foreach form, amsgrad off):
//   p *= 1 - lr wd;  m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g g
//   p += -step_size * m / (sqrt(v) / bc2_sqrt + eps)
__global__ void __launch_bounds__(kThreads)
adamw_kernel(const Slot* __restrict__ slots, int nslots, long long total, float decay, float w1, float beta2,
             float omb2, float bc2_sqrt, float eps, float neg_step) {
  for_each_elem(slots, nslots, total, [&](const Slot& s, long long i) {
    const float g = s.grad[i];
    float p = s.param[i] * decay;
    float m = s.exp_avg[i];
    m = m + w1 * (g - m);                      // lerp, weight < 0.5 branch
    float v = s.exp_avg_sq[i] * beta2;
    v = v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + neg_step * m / denom;
    s.param[i] = p;
    s.exp_avg[i] = m;
    s.exp_avg_sq[i] = v;
  });
}

// 16-bit parameters and state (a model.to(bfloat16) / .half() run): the same update with
// every foreach op's result stored in T, as torch's _multi_tensor_adam (decoupled weight
// decay) does: each _foreach_* call computes in fp32 and writes T
template <typename T>
__global__ void __launch_bounds__(kThreads)
adamw16_kernel(const Slot* __restrict__ slots, int nslots, long long total, float decay, float w1, float beta2,
               float omb2, float bc2_sqrt, float eps, float neg_step) {
#pragma clang fp contract(off)
  for_each_elem(slots, nslots, total, [&](const Slot& s, long long i) {
    T* P = reinterpret_cast<T*>(s.param);
    T* M = reinterpret_cast<T*>(s.exp_avg);
    T* V = reinterpret_cast<T*>(s.exp_avg_sq);
    const float g = (float)reinterpret_cast<const T*>(s.grad)[i];
    // ATen's device functors contract a + b * c into one fma (the compiler's default); the
    // same contractions here, explicitly, everything else one rounding per op
    const float p = rt<T>((float)P[i] * decay);                         // _foreach_mul_(params, 1 - lr wd)
    const float m0 = (float)M[i];
    const float m = rt<T>(w1 < 0.5f ? fmaf(w1, g - m0, m0) : fmaf(-(g - m0), 1.f - w1, g));   // _foreach_lerp_
    float v = rt<T>((float)V[i] * beta2);                               // _foreach_mul_(v, b2)
    v = rt<T>(fmaf(omb2 * g, g, v));                                    // _foreach_addcmul_(v, g, g, 1 - b2)
    float d = rt<T>(sqrtf(v));                                          // _foreach_sqrt
    d = rt<T>(d / bc2_sqrt);                                            // _foreach_div_
    d = rt<T>(d + eps);                                                 // _foreach_add_
    P[i] = (T)fmaf(neg_step, m / d, p);                                 // _foreach_addcdiv_
    M[i] = (T)m;
    V[i] = (T)v;
  });
}

constexpr int kMaxSlotGrid = 2048;
inline unsigned slot_grid(long long total) {
  const long long g = (total + kChunk - 1) / kChunk;
  return (unsigned)(g < kMaxSlotGrid ? (g > 0 ? g : 1) : kMaxSlotGrid);
}

}  // namespace

extern "C" size_t se_sisnr_save_bytes(int B) { return (size_t)(B > 0 ? B : 0) * kSave * sizeof(double); }

#define SE_DT_SWITCH(dtype, BODY)                  \
  switch (dtype) {                                 \
    case SE_DTYPE_F32: { using TY = float; BODY; } break;    \
    case SE_DTYPE_BF16: { using TY = __bf16; BODY; } break;  \
    case SE_DTYPE_F16: { using TY = _Float16; BODY; } break; \
    default: return SE_E_ARG;                      \
  }

extern "C" int se_sisnr_fwd(const void* est, int le, long long est_stride, const void* target, int lt, int B,
                            int zero_mean, float eps, void* loss, void* save, int dtype, void* stream) {
  if (!est || !target || !loss || !save || B <= 0 || le <= 0 || lt <= 0 || est_stride < le) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(sisnr_items_kernel<TY>, dim3(B), dim3(kItemThreads), 0, st, (const TY*)est, le, est_stride,
                       (const TY*)target, lt, zero_mean, (double*)save);
    SE_LAUNCH_CHECK();
    hipLaunchKernelGGL(sisnr_finalize_kernel<TY>, dim3(1), dim3(kThreads), 0, st, (const double*)save, B, eps,
                       (TY*)loss);
    SE_LAUNCH_CHECK();
  })
  return SE_OK;
}

extern "C" int se_sisnr_bwd(const void* est, int le, long long est_stride, const void* target, int lt, int B,
                            int zero_mean, float eps, const void* save, const void* grad_loss, void* grad_est,
                            long long grad_stride, int dtype, void* stream) {
  if (!est || !target || !save || !grad_loss || !grad_est || B <= 0 || le <= 0 || lt <= 0 || est_stride < le ||
      grad_stride < le)
    return SE_E_ARG;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(sisnr_bwd_kernel<TY>, dim3(se::ceil_div(le, 4 * kThreads), B), dim3(kThreads), 0,
                       se::as_stream(stream), (const TY*)est, le, est_stride, (const TY*)target, lt, B, zero_mean,
                       eps, (const double*)save, (const TY*)grad_loss, (TY*)grad_est, grad_stride);
    SE_LAUNCH_CHECK();
  })
  return SE_OK;
}

extern "C" int se_grad_sumsq(const se_tensor_slot* slots, int nslots, long long total, double* sumsq, int dtype,
                             void* stream) {
  if (!slots || !sumsq || nslots <= 0 || total < 0) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  if (total == 0) return hipMemsetAsync(sumsq, 0, sizeof(double), st) == hipSuccess ? SE_OK : SE_E_LAUNCH;
  const unsigned grid = slot_grid(total);
  static_assert(kMaxSlotGrid + 1 == SE_SUMSQ_DOUBLES, "partials fit the caller's buffer");
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(sumsq_kernel<TY>, dim3(grid), dim3(kThreads), 0, st, (const Slot*)slots, nslots, total,
                       sumsq);
  })
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(kThreads), 0, st, sumsq, (int)grid);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_clip_grads(const se_tensor_slot* slots, int nslots, long long total, const double* sumsq,
                             float max_norm, float* total_norm, int dtype, void* stream) {
  if (!slots || !sumsq || nslots <= 0 || total < 0) return SE_E_ARG;
  if (total == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(clip_kernel<TY>, dim3(slot_grid(total)), dim3(kThreads), 0, se::as_stream(stream),
                       (const Slot*)slots, nslots, total, sumsq, max_norm, total_norm);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_adamw_step(const se_tensor_slot* slots, int nslots, long long total, double lr, double beta1,
                             double beta2, double eps, double weight_decay, long long step, int dtype, void* stream) {
  if (!slots || nslots <= 0 || total < 0 || step < 1) return SE_E_ARG;
  if (total == 0) return SE_OK;
  // host scalars as torch computes them (Python floats, then the kernel's fp32)
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float a0 = (float)(1.0 - lr * weight_decay), a1 = (float)(1.0 - beta1), a2 = (float)beta2,
              a3 = (float)(1.0 - beta2), a4 = (float)std::sqrt(bc2), a5 = (float)eps, a6 = (float)(-(lr / bc1));
  hipStream_t st = se::as_stream(stream);
  const dim3 grid(slot_grid(total));
  switch (dtype) {
    case SE_DTYPE_F32:
      hipLaunchKernelGGL(adamw_kernel, grid, dim3(kThreads), 0, st, (const Slot*)slots, nslots, total, a0, a1, a2,
                         a3, a4, a5, a6);
      break;
    case SE_DTYPE_BF16:
      hipLaunchKernelGGL(adamw16_kernel<__bf16>, grid, dim3(kThreads), 0, st, (const Slot*)slots, nslots, total, a0,
                         a1, a2, a3, a4, a5, a6);
      break;
    case SE_DTYPE_F16:
      hipLaunchKernelGGL(adamw16_kernel<_Float16>, grid, dim3(kThreads), 0, st, (const Slot*)slots, nslots, total,
                         a0, a1, a2, a3, a4, a5, a6);
      break;
    default: return SE_E_ARG;
  }
  SE_LAUNCH_CHECK();
  return SE_OK;
}

// ------------------------------------------------------------------ FRCRN mask
// frcrn.py:140-152: mask = tanh(pad(h, top 1 row)); est = pad(mask * noisy, top 1)
// with noisy = the spectrum without its DC row, re-stacked as [B, 2*half, T]. So
//   est[b, c*half + k, t] = k < 2 ? 0 : tanh(h[b, c, k - 2, t]) * spec[b, c*half + k, t]
// (row 0: the DC re-padded as 0; row 1: tanh(0) = 0 from the mask pad). One pass
// instead of pad / tanh / mul / pad / reshape; the backward is one pass too:
//   dh[b, c, k - 2, t] = dest * spec * (1 - tanh^2)   (the spectrum takes no gradient).
// grid (ceil(half * T / (4 kThreads)), 2 B)
__global__ void __launch_bounds__(kThreads)
mask_fwd_kernel(const float* __restrict__ h, const float* __restrict__ spec, int half, int T,
                float* __restrict__ est) {
  const int bc = blockIdx.y;                     // b * 2 + c
  const long long HT = (long long)half * T;
  const float* hp = h + (long long)bc * (half - 2) * T;
  const float* sp = spec + (long long)bc * HT;
  float* ep = est + (long long)bc * HT;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = ((long long)blockIdx.x * 4 + u) * kThreads + threadIdx.x;
    if (i >= HT) return;
    const long long k = i / T;
    ep[i] = k < 2 ? 0.f : tanhf(hp[i - 2 * T]) * sp[i];
  }
}

__global__ void __launch_bounds__(kThreads)
mask_bwd_kernel(const float* __restrict__ gest, const float* __restrict__ h, const float* __restrict__ spec,
                int half, int T, float* __restrict__ gh) {
  const int bc = blockIdx.y;
  const long long HT = (long long)half * T, HT2 = (long long)(half - 2) * T;
  const float* hp = h + (long long)bc * HT2;
  const float* sp = spec + (long long)bc * HT + 2 * T;
  const float* gp = gest + (long long)bc * HT + 2 * T;
  float* op = gh + (long long)bc * HT2;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = ((long long)blockIdx.x * 4 + u) * kThreads + threadIdx.x;
    if (i >= HT2) return;
    const float m = tanhf(hp[i]);
    op[i] = gp[i] * sp[i] * (1.f - m * m);
  }
}

// Magnitude / phase masks of the inference forward (no gradient), one pass instead of the
// reference's ~20 elementwise kernels:
//   mode 0, DCUNet bounded_tanh (_1903_03107_dcunet.py:167-189):
//     ph = n_ph + m_ph / m_mag, gain = n_mag * tanh(m_mag)
//   mode 1, DCCRN 'E' (_2008_00264_dccrn.py:194-207):
//     m_ph = atan2(mi / m_mag, mr / m_mag), ph = n_ph + m_ph, gain = n_mag * tanh(m_mag)
// with mag = sqrt(re^2 + im^2 + 1e-8), phase = atan2(im, re); out = gain * (cos ph, sin ph)
// into [B, 2, F, T]. Each intermediate is rounded to the storage type T exactly where the
// reference's tensors are (a bf16 / fp16 model computes every op in fp32 and stores T), in the
// reference's operation order without contraction; the transcendental functions are this
// toolchain's (torch's build may differ in the last ulp, which the phase terms can amplify).
// m / n rows: batch stride, row stride (elements), time contiguous. grid (ceil(F T / 256), B)
template <typename T, int MODE>
__global__ void __launch_bounds__(kThreads)
polar_mask_fwd_kernel(const T* __restrict__ mr, const T* __restrict__ mi, long long msb, long long msr,
                      const T* __restrict__ nr, const T* __restrict__ ni, long long nsb, long long nsr, int F, int Tn,
                      int row0, T* __restrict__ out) {
#pragma clang fp contract(off)   // one rounding per reference op: no fused multiply-adds
  const int b = blockIdx.y;
  const long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= (long long)F * Tn) return;
  const int f = (int)(i / Tn), t = (int)(i - (long long)f * Tn);
  const long long mo = b * msb + (long long)(f - row0) * msr + t, no = b * nsb + f * nsr + t;
  const bool mz = f < row0;   // a leading zero row of the mask (not stored)
  const float a = mz ? 0.f : (float)mr[mo], c = mz ? 0.f : (float)mi[mo], x = (float)nr[no], y = (float)ni[no];
  auto mag = [](float re, float im) __attribute__((always_inline)) {
    return rt<T>(sqrtf(rt<T>(rt<T>(rt<T>(re * re) + rt<T>(im * im)) + 1e-8f)));
  };
  const float m_mag = mag(a, c), n_mag = mag(x, y);
  const float n_ph = rt<T>(atan2f(y, x));
  float ph;
  if constexpr (MODE == 0) {
    const float m_ph = rt<T>(atan2f(c, a));
    ph = rt<T>(n_ph + rt<T>(m_ph / m_mag));
  } else {
    const float m_ph = rt<T>(atan2f(rt<T>(c / m_mag), rt<T>(a / m_mag)));
    ph = rt<T>(n_ph + m_ph);
  }
  const float gain = rt<T>(n_mag * rt<T>(tanhf(m_mag)));
  const long long oo = (long long)b * 2 * F * Tn + i;
  out[oo] = (T)(gain * rt<T>(cosf(ph)));
  out[oo + (long long)F * Tn] = (T)(gain * rt<T>(sinf(ph)));
}

extern "C" int se_polar_mask_fwd(const void* mr, const void* mi, long long m_batch_stride, long long m_row_stride,
                                 const void* nr, const void* ni, long long n_batch_stride, long long n_row_stride,
                                 int B, int F, int T, int mode, int dtype, int m_row0, void* out, void* stream) {
  if (!mr || !mi || !nr || !ni || !out || B <= 0 || F <= 0 || T <= 0 || (mode != 0 && mode != 1) || m_row0 < 0 ||
      m_row0 >= F)
    return SE_E_ARG;
  const dim3 grid((unsigned)se::ceil_div((long long)F * T, kThreads), B);
  hipStream_t st = se::as_stream(stream);
#define SE_PM(TY)                                                                                                  \
  do {                                                                                                             \
    if (mode == 0)                                                                                                 \
      hipLaunchKernelGGL((polar_mask_fwd_kernel<TY, 0>), grid, dim3(kThreads), 0, st, (const TY*)mr, (const TY*)mi, \
                         m_batch_stride, m_row_stride, (const TY*)nr, (const TY*)ni, n_batch_stride, n_row_stride, F, \
                         T, m_row0, (TY*)out);                                                                          \
    else                                                                                                           \
      hipLaunchKernelGGL((polar_mask_fwd_kernel<TY, 1>), grid, dim3(kThreads), 0, st, (const TY*)mr, (const TY*)mi, \
                         m_batch_stride, m_row_stride, (const TY*)nr, (const TY*)ni, n_batch_stride, n_row_stride, F, \
                         T, m_row0, (TY*)out);                                                                          \
  } while (0)
  switch (dtype) {
    case SE_DTYPE_F32: SE_PM(float); break;
    case SE_DTYPE_BF16: SE_PM(__bf16); break;
    case SE_DTYPE_F16: SE_PM(_Float16); break;
    default: return SE_E_ARG;
  }
#undef SE_PM
  SE_LAUNCH_CHECK();
  return SE_OK;
}

// Backward of the masks above for a training forward (the mask takes the gradient, the
// noisy spectrum none): from g = dL/d(re, im) [B, 2, F, T],
//   d_gain = g_re cos ph + g_im sin ph,   d_ph = gain (g_im cos ph - g_re sin ph)
//   d_mag  = d_gain n_mag (1 - tanh^2 m_mag)  (+ the phase path's m_mag terms)
// through atan2 (d/dy = x / (x^2 + y^2), d/dx = -y / (x^2 + y^2), 0 where x^2 + y^2 == 0, as
// torch's atan2 backward)
// and m_mag = sqrt(mr^2 + mi^2 + 1e-8) (d/dmr = mr / m_mag). fp32 arithmetic on the storage
// values, the forward's intermediates recomputed (T-rounded as in the forward), gradients
// rounded to T once. dm [B, 2, F, T]: (d mr, d mi).
template <typename T, int MODE>
__global__ void __launch_bounds__(kThreads)
polar_mask_bwd_kernel(const T* __restrict__ g, const T* __restrict__ mr, const T* __restrict__ mi, long long msb,
                      long long msr, const T* __restrict__ nr, const T* __restrict__ ni, long long nsb, long long nsr,
                      int F, int Tn, int row0, int dmT, T* __restrict__ dm) {
#pragma clang fp contract(off)
  const int b = blockIdx.y;
  const long long Fd = F - row0, i = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= Fd * dmT) return;
  const int fd = (int)(i / dmT), t = (int)(i - (long long)fd * dmT), f = fd + row0;
  const long long od = (long long)b * 2 * Fd * dmT + i;
  if (t >= Tn) {   // a trimmed frame of the stored mask: no gradient
    dm[od] = (T)0.f;
    dm[od + Fd * dmT] = (T)0.f;
    return;
  }
  const long long mo = b * msb + (long long)fd * msr + t, no = b * nsb + f * nsr + t;
  const float a = (float)mr[mo], c = (float)mi[mo], x = (float)nr[no], y = (float)ni[no];
  auto mag = [](float re, float im) __attribute__((always_inline)) {
    return rt<T>(sqrtf(rt<T>(rt<T>(rt<T>(re * re) + rt<T>(im * im)) + 1e-8f)));
  };
  const float m_mag = mag(a, c), n_mag = mag(x, y);
  const float n_ph = rt<T>(atan2f(y, x));
  const float th = rt<T>(tanhf(m_mag));
  const float gain = rt<T>(n_mag * th);
  float ph, m_ph, u = 0.f, v = 0.f;
  if constexpr (MODE == 0) {
    m_ph = rt<T>(atan2f(c, a));
    ph = rt<T>(n_ph + rt<T>(m_ph / m_mag));
  } else {
    u = rt<T>(a / m_mag);
    v = rt<T>(c / m_mag);
    m_ph = rt<T>(atan2f(v, u));
    ph = rt<T>(n_ph + m_ph);
  }
  const long long FT = (long long)F * Tn, oo = (long long)b * 2 * FT + (long long)f * Tn + t;
  const float gre = (float)g[oo], gim = (float)g[oo + FT];
  // the forward's T-rounded cos / sin factors (torch's mul backward reads the stored factor)
  const float cp = rt<T>(cosf(ph)), sp = rt<T>(sinf(ph));
  const float d_gain = gre * cp + gim * sp;
  const float d_ph = gain * (gim * cp - gre * sp);
  float d_mag = d_gain * n_mag * (1.f - th * th);
  float da, dc;
  // torch's atan2 backward is 0 where x^2 + y^2 == 0 (the origin, or squares that underflow)
  if constexpr (MODE == 0) {
    const float d_mph = d_ph / m_mag;                 // ph = n_ph + m_ph / m_mag
    d_mag += d_ph * (-m_ph / (m_mag * m_mag));
    const float r2 = a * a + c * c;
    da = r2 == 0.f ? 0.f : d_mph * (-c / r2);
    dc = r2 == 0.f ? 0.f : d_mph * (a / r2);
  } else {
    const float r2 = u * u + v * v;                   // m_ph = atan2(v, u), u = mr / m_mag, v = mi / m_mag
    const float du = r2 == 0.f ? 0.f : d_ph * (-v / r2), dv = r2 == 0.f ? 0.f : d_ph * (u / r2);
    d_mag += du * (-a / (m_mag * m_mag)) + dv * (-c / (m_mag * m_mag));
    da = du / m_mag;
    dc = dv / m_mag;
  }
  da += d_mag * (a / m_mag);
  dc += d_mag * (c / m_mag);
  dm[od] = (T)da;
  dm[od + Fd * dmT] = (T)dc;
}

extern "C" int se_polar_mask_bwd(const void* g, const void* mr, const void* mi, long long m_batch_stride,
                                 long long m_row_stride, const void* nr, const void* ni, long long n_batch_stride,
                                 long long n_row_stride, int B, int F, int T, int mode, int dtype, int m_row0,
                                 int dm_T, void* dm, void* stream) {
  if (!g || !mr || !mi || !nr || !ni || !dm || B <= 0 || F <= 0 || T <= 0 || (mode != 0 && mode != 1) ||
      m_row0 < 0 || m_row0 >= F || dm_T < T)
    return SE_E_ARG;
  const dim3 grid((unsigned)se::ceil_div((long long)(F - m_row0) * dm_T, kThreads), B);
  hipStream_t st = se::as_stream(stream);
#define SE_PMB(TY)                                                                                                 \
  do {                                                                                                             \
    if (mode == 0)                                                                                                 \
      hipLaunchKernelGGL((polar_mask_bwd_kernel<TY, 0>), grid, dim3(kThreads), 0, st, (const TY*)g, (const TY*)mr,  \
                         (const TY*)mi, m_batch_stride, m_row_stride, (const TY*)nr, (const TY*)ni, n_batch_stride, \
                         n_row_stride, F, T, m_row0, dm_T, (TY*)dm);                                                          \
    else                                                                                                           \
      hipLaunchKernelGGL((polar_mask_bwd_kernel<TY, 1>), grid, dim3(kThreads), 0, st, (const TY*)g, (const TY*)mr,  \
                         (const TY*)mi, m_batch_stride, m_row_stride, (const TY*)nr, (const TY*)ni, n_batch_stride, \
                         n_row_stride, F, T, m_row0, dm_T, (TY*)dm);                                                          \
  } while (0)
  switch (dtype) {
    case SE_DTYPE_F32: SE_PMB(float); break;
    case SE_DTYPE_BF16: SE_PMB(__bf16); break;
    case SE_DTYPE_F16: SE_PMB(_Float16); break;
    default: return SE_E_ARG;
  }
#undef SE_PMB
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_mask_fwd(const float* h, const float* spec, int B, int half, int T, float* est, void* stream) {
  if (!h || !spec || !est || B <= 0 || half < 3 || T <= 0) return SE_E_ARG;
  hipLaunchKernelGGL(mask_fwd_kernel, dim3(se::ceil_div((long long)half * T, 4 * kThreads), 2 * B), dim3(kThreads), 0,
                     se::as_stream(stream), h, spec, half, T, est);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_mask_bwd(const float* gest, const float* h, const float* spec, int B, int half, int T, float* gh,
                           void* stream) {
  if (!gest || !h || !spec || !gh || B <= 0 || half < 3 || T <= 0) return SE_E_ARG;
  hipLaunchKernelGGL(mask_bwd_kernel, dim3(se::ceil_div((long long)(half - 2) * T, 4 * kThreads), 2 * B),
                     dim3(kThreads), 0, se::as_stream(stream), gest, h, spec, half, T, gh);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
