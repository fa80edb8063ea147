// The models' glue around the GEMMs, as HIP passes (ABI 10): the layout changes
// and casts the reference writes as .contiguous() / .float() / cat / chunk, the
// ComplexLSTM re / im combination, a Linear's bias gradient over any layout,
// CARN's attention gates, mask and clamp, and the long-form chunking. All of
// it is HBM-bound elementwise or reduction work: coalesced along the innermost
// index, fp32 arithmetic, storage type T (fp32 / bf16 / fp16) rounded where the
// reference's tensors are.
#include "common.hpp"

namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ float rt(float v) { return (float)(T)v; }
__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + __expf(-z)); }

#define SE_DT_SWITCH(dtype, BODY)                              \
  switch (dtype) {                                             \
    case SE_DTYPE_F32: { using TY = float; BODY; } break;      \
    case SE_DTYPE_BF16: { using TY = __bf16; BODY; } break;    \
    case SE_DTYPE_F16: { using TY = _Float16; BODY; } break;   \
    default: return SE_E_ARG;                                  \
  }

inline unsigned grid_of(long long n, int per_thread = 1) {
  const long long g = (n + (long long)kThreads * per_thread - 1) / ((long long)kThreads * per_thread);
  return (unsigned)(g < 65535LL * 16 ? (g > 0 ? g : 1) : 65535LL * 16);
}

// ------------------------------------------------------------------ strided copy
struct CopyDims {
  long long size[SE_COPY_MAX_DIMS];
  long long ss[SE_COPY_MAX_DIMS];   // source strides
  long long ds[SE_COPY_MAX_DIMS];   // destination strides
  int nd;
  long long total;
};

// one element per thread-iteration, the flat index decomposed innermost-first (the
// host orders the dims so the innermost one is the contiguous side of the larger tensor)
template <typename S, typename D>
__global__ void __launch_bounds__(kThreads) copy_strided_kernel(const S* __restrict__ src, D* __restrict__ dst,
                                                                const CopyDims d) {
  for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < d.total;
       idx += (long long)gridDim.x * kThreads) {
    long long r = idx, so = 0, dof = 0;
#pragma unroll
    for (int k = SE_COPY_MAX_DIMS - 1; k >= 0; --k) {
      if (k >= d.nd) continue;
      const long long q = r / d.size[k];
      const long long i = r - q * d.size[k];
      r = q;
      so += i * d.ss[k];
      dof += i * d.ds[k];
    }
    dst[dof] = (D)(float)src[so];
  }
}

// ------------------------------------------------------------------ bias gradient
constexpr int kColChunks = 64;
// sg == 1 (dy rows of G contiguous values): chunks of rows summed in row order per column,
// then the chunk partials in order (grid: ceil(G / 256) x kColChunks)
template <typename T>
__global__ void __launch_bounds__(kThreads) bias_col_part_kernel(const T* __restrict__ x, int L, long long R, int G,
                                                                 long long sl, long long sr, float* __restrict__ part) {
  const int g = blockIdx.x * kThreads + threadIdx.x, ch = blockIdx.y;
  if (g >= G) return;
  const long long LR = (long long)L * R, rows = (LR + kColChunks - 1) / kColChunks;
  const long long r0 = (long long)ch * rows, r1 = min(LR, r0 + rows);
  float s = 0.f;
  for (long long q = r0; q < r1; ++q) {
    const long long l = q / R, r = q - l * R;
    s += (float)x[l * sl + r * sr + g];
  }
  part[(long long)ch * G + g] = s;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) bias_col_final_kernel(const float* __restrict__ part, int G,
                                                                  T* __restrict__ out) {
  const int g = blockIdx.x * kThreads + threadIdx.x;
  if (g >= G) return;
  float s = 0.f;
#pragma unroll 8
  for (int c = 0; c < kColChunks; ++c) s += part[(long long)c * G + g];
  out[g] = (T)s;
}

// general strides (sr == 1: contiguous rows per g): one workgroup per g, lanes over r
template <typename T>
__global__ void __launch_bounds__(kThreads) bias_row_kernel(const T* __restrict__ x, int L, long long R,
                                                            long long sl, long long sr, long long sg,
                                                            T* __restrict__ out) {
  const int g = blockIdx.x;
  __shared__ float red[kThreads / 64];
  float s = 0.f;
  for (int l = 0; l < L; ++l) {
    const T* p = x + l * sl + g * sg;
    for (long long r = threadIdx.x; r < R; r += kThreads) s += (float)p[r * sr];
  }
  s = se::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[g] = (T)(red[0] + red[1] + red[2] + red[3]);
}

// ------------------------------------------------------------------ ComplexLSTM combine
// out[b, t, k] = k < H ? h0[b] - h1[B + b] : h1[b] + h0[B + b]  (complex_nn.py:134-142);
// the flat index runs k fastest for a feature-contiguous out (osk == 1), else t fastest, so
// the stores stay coalesced either way
template <typename T>
__global__ void __launch_bounds__(kThreads) clstm_combine_fwd_kernel(const float* __restrict__ h, long long hls,
                                                                     int B, int Tn, int H, T* __restrict__ out,
                                                                     long long osb, long long osr, long long osk) {
  const long long total = (long long)B * Tn * 2 * H;
  const long long half_b = (long long)B * Tn * H;   // offset of batch row B within one LSTM's h
  const bool kfast = osk == 1;
  for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * kThreads) {
    int b, t, k;
    if (kfast) {
      k = (int)(idx % (2 * H));
      const long long bt = idx / (2 * H);
      b = (int)(bt / Tn);
      t = (int)(bt - (long long)b * Tn);
    } else {
      t = (int)(idx % Tn);
      const long long bk = idx / Tn;
      b = (int)(bk / (2 * H));
      k = (int)(bk - (long long)b * 2 * H);
    }
    const int kk = k < H ? k : k - H;
    const long long o = ((long long)b * Tn + t) * H + kk;
    float v;
    if (k < H) v = h[o] - h[hls + half_b + o];
    else v = h[hls + o] + h[half_b + o];
    out[b * osb + t * osr + k * osk] = (T)v;
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) clstm_combine_bwd_kernel(const T* __restrict__ g, long long gsb,
                                                                     long long gsr, long long gsk, int B, int Tn,
                                                                     int H, float* __restrict__ dh, long long hls) {
  const long long total = (long long)B * Tn * H;
  for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * kThreads) {
    const int k = (int)(idx % H);
    const long long bt = idx / H;
    const int b = (int)(bt / Tn), t = (int)(bt - (long long)b * Tn);
    const long long gi = b * gsb + t * gsr + k * gsk;
    const float gre = (float)g[gi], gim = (float)g[gi + H * gsk];
    dh[idx] = gre;                       // real_lstm(re)
    dh[hls + total + idx] = -gre;        // imag_lstm(im)
    dh[hls + idx] = gim;                 // imag_lstm(re)
    dh[total + idx] = gim;               // real_lstm(im)
  }
}

// ------------------------------------------------------------------ CARN
// est[b, f] = mr nr - mi ni, est[b, half + f] = mr ni - mi nr  (carn.py:161-168)
template <typename T>
__global__ void __launch_bounds__(kThreads) carn_mask_fwd_kernel(const T* __restrict__ m, long long msb,
                                                                 const T* __restrict__ spec, int half, int Tn,
                                                                 T* __restrict__ est) {
#pragma clang fp contract(off)
  const int b = blockIdx.y;
  const long long HT = (long long)half * Tn;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < HT; i += (long long)gridDim.x * kThreads) {
    const float mr = (float)m[b * msb + i], mi = (float)m[b * msb + HT + i];
    const float nr = (float)spec[(long long)b * 2 * HT + i], ni = (float)spec[(long long)b * 2 * HT + HT + i];
    est[(long long)b * 2 * HT + i] = (T)(rt<T>(mr * nr) - rt<T>(mi * ni));
    est[(long long)b * 2 * HT + HT + i] = (T)(rt<T>(mr * ni) - rt<T>(mi * nr));
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) carn_mask_bwd_kernel(const T* __restrict__ g, const T* __restrict__ m,
                                                                 long long msb, const T* __restrict__ spec, int half,
                                                                 int Tn, T* __restrict__ dm, T* __restrict__ dspec) {
  const int b = blockIdx.y;
  const long long HT = (long long)half * Tn;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < HT; i += (long long)gridDim.x * kThreads) {
    const long long so = (long long)b * 2 * HT + i;
    const float gr = (float)g[so], gi = (float)g[so + HT];
    const float nr = (float)spec[so], ni = (float)spec[so + HT];
    const float mr = (float)m[b * msb + i], mi = (float)m[b * msb + HT + i];
    dm[so] = (T)(gr * nr + gi * ni);
    dm[so + HT] = (T)(-gr * ni - gi * nr);
    if (dspec) {
      dspec[so] = (T)(gr * mr - gi * mi);
      dspec[so + HT] = (T)(gi * mr - gr * mi);
    }
  }
}

// y = sigmoid(a + b)   (carn.py:70-72)
template <typename T>
__global__ void __launch_bounds__(kThreads) add_sigmoid_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                               T* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    y[i] = (T)sigm(rt<T>((float)a[i] + (float)b[i]));
}

template <typename T>
__global__ void __launch_bounds__(kThreads) sigmoid_kernel(const T* __restrict__ x, T* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    y[i] = (T)(1.f / (1.f + expf(-(float)x[i])));
}

// dz = g (1 - y) y   (torch's sigmoid_backward)
template <typename T>
__global__ void __launch_bounds__(kThreads) sigmoid_bwd_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                               T* __restrict__ dz, long long n) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const float yv = (float)y[i];
    dz[i] = (T)((float)g[i] * (1.f - yv) * yv);
  }
}

// out[b, 0:C] = sigmoid(c) * skip, out[b, C:2C] = skip   (carn.py:74-76, :112-113)
template <typename T>
__global__ void __launch_bounds__(kThreads) gate_cat_fwd_kernel(const T* __restrict__ c, const T* __restrict__ skip,
                                                                T* __restrict__ out, long long CHW) {
  const int b = blockIdx.y;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < CHW; i += (long long)gridDim.x * kThreads) {
    const long long o = (long long)b * CHW + i;
    const float s = (float)skip[o];
    out[2 * (long long)b * CHW + i] = (T)(rt<T>(sigm((float)c[o])) * s);
    out[2 * (long long)b * CHW + CHW + i] = (T)s;
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) gate_cat_bwd_kernel(const T* __restrict__ g, const T* __restrict__ c,
                                                                const T* __restrict__ skip, T* __restrict__ dc,
                                                                T* __restrict__ dskip, long long CHW) {
  const int b = blockIdx.y;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < CHW; i += (long long)gridDim.x * kThreads) {
    const long long o = (long long)b * CHW + i;
    const float g0 = (float)g[2 * (long long)b * CHW + i], g1 = (float)g[2 * (long long)b * CHW + CHW + i];
    const float sg = rt<T>(sigm((float)c[o])), s = (float)skip[o];
    dskip[o] = (T)(g1 + g0 * sg);
    dc[o] = (T)(rt<T>(g0 * s) * (1.f - sg) * sg);
  }
}

// y = a * sigmoid(b)   (ConvGLU / DeConvGLU, carn.py:9-27)
template <typename T>
__global__ void __launch_bounds__(kThreads) glu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                           T* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    y[i] = (T)((float)a[i] * rt<T>(sigm((float)b[i])));
}

template <typename T>
__global__ void __launch_bounds__(kThreads) glu_bwd_kernel(const T* __restrict__ g, const T* __restrict__ a,
                                                           const T* __restrict__ b, T* __restrict__ da,
                                                           T* __restrict__ db, long long n) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const float gv = (float)g[i], s = rt<T>(sigm((float)b[i]));
    da[i] = (T)(gv * s);
    db[i] = (T)(rt<T>(gv * (float)a[i]) * (1.f - s) * s);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) clamp_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long long n,
                                                             float lo, float hi) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    y[i] = (T)fminf(fmaxf((float)x[i], lo), hi);
}

template <typename T>
__global__ void __launch_bounds__(kThreads) clamp_bwd_kernel(const T* __restrict__ g, const T* __restrict__ x,
                                                             T* __restrict__ dx, long long n, float lo, float hi) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const float v = (float)x[i];
    dx[i] = (v >= lo && v <= hi) ? g[i] : (T)0.f;
  }
}

// ------------------------------------------------------------------ long-form chunking
template <typename T>
__global__ void __launch_bounds__(kThreads) chunk_split_kernel(const T* __restrict__ x, long long L, int chunk,
                                                               int hop, T* __restrict__ out, long long total) {
  for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * kThreads) {
    const long long i = idx / chunk, s = idx - i * chunk, p = i * hop + s;
    out[idx] = p < L ? x[p] : (T)0.f;
  }
}

// the chunk weights of sehip/longform.py's overlap_add, in T: ramp (j + 0.5) / overlap
// computed in fp32 and rounded (ramp.to(dtype)), fade-out 1 - ramp likewise
template <typename T>
__global__ void __launch_bounds__(kThreads) chunk_ola_kernel(const T* __restrict__ y, int n, int width, int chunk,
                                                             int overlap, long long length, T* __restrict__ out) {
#pragma clang fp contract(off)
  const int hop = chunk - overlap;
  for (long long p = (long long)blockIdx.x * kThreads + threadIdx.x; p < length;
       p += (long long)gridDim.x * kThreads) {
    long long i0 = p >= chunk ? (p - chunk) / hop + 1 : 0;   // first chunk covering p
    long long i1 = p / hop;                                   // last chunk starting at or before p
    if (i1 > n - 1) i1 = n - 1;
    float acc = 0.f;
    for (long long i = i0; i <= i1; ++i) {
      const int s = (int)(p - i * hop);
      if (s < 0 || s >= chunk) continue;
      float v = s < width ? (float)y[i * width + s] : 0.f;
      float w = 1.f;   // the fade-out is assigned last in the reference loop: it wins where both apply
      if (overlap && i > 0 && s < overlap) w = rt<T>(((float)s + 0.5f) / (float)overlap);
      if (overlap && i < n - 1 && s >= chunk - overlap) {
        const int j = s - (chunk - overlap);
        w = rt<T>(1.f - ((float)j + 0.5f) / (float)overlap);
      }
      acc = rt<T>(acc + rt<T>(v * w));
    }
    out[p] = (T)acc;
  }
}

}  // namespace

extern "C" int se_copy_strided(const void* src, int src_dtype, void* dst, int dst_dtype, int ndim,
                               const long long* sizes, const long long* src_strides, const long long* dst_strides,
                               void* stream) {
  if (!src || !dst || !sizes || !src_strides || !dst_strides || ndim < 1 || ndim > SE_COPY_MAX_DIMS) return SE_E_ARG;
  CopyDims d{};
  d.nd = ndim;
  d.total = 1;
  for (int k = 0; k < ndim; ++k) {
    if (sizes[k] < 0) return SE_E_ARG;
    d.size[k] = sizes[k] ? sizes[k] : 1;
    d.ss[k] = src_strides[k];
    d.ds[k] = dst_strides[k];
    d.total *= sizes[k];
  }
  if (d.total == 0) return SE_OK;
  hipStream_t st = se::as_stream(stream);
  const unsigned grid = grid_of(d.total, 4);
#define SE_CP(S)                                                                                                  \
  switch (dst_dtype) {                                                                                            \
    case SE_DTYPE_F32:                                                                                            \
      hipLaunchKernelGGL((copy_strided_kernel<S, float>), dim3(grid), dim3(kThreads), 0, st, (const S*)src,       \
                         (float*)dst, d);                                                                         \
      break;                                                                                                      \
    case SE_DTYPE_BF16:                                                                                           \
      hipLaunchKernelGGL((copy_strided_kernel<S, __bf16>), dim3(grid), dim3(kThreads), 0, st, (const S*)src,      \
                         (__bf16*)dst, d);                                                                        \
      break;                                                                                                      \
    case SE_DTYPE_F16:                                                                                            \
      hipLaunchKernelGGL((copy_strided_kernel<S, _Float16>), dim3(grid), dim3(kThreads), 0, st, (const S*)src,    \
                         (_Float16*)dst, d);                                                                      \
      break;                                                                                                      \
    default: return SE_E_ARG;                                                                                     \
  }
  switch (src_dtype) {
    case SE_DTYPE_F32: SE_CP(float); break;
    case SE_DTYPE_BF16: SE_CP(__bf16); break;
    case SE_DTYPE_F16: SE_CP(_Float16); break;
    default: return SE_E_ARG;
  }
#undef SE_CP
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" size_t se_bias_grad_workspace_size(int L, long long R, int G) {
  if (L <= 0 || R <= 0 || G <= 0) return 0;
  return (size_t)kColChunks * G * sizeof(float);
}

extern "C" int se_bias_grad(const void* x, int L, long long R, int G, long long sl, long long sr, long long sg,
                            int dtype, void* out, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !out || L <= 0 || R <= 0 || G <= 0) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  if (sg == 1) {
    if (!ws || ws_bytes < se_bias_grad_workspace_size(L, R, G)) return SE_E_WORKSPACE;
    SE_DT_SWITCH(dtype, {
      hipLaunchKernelGGL(bias_col_part_kernel<TY>, dim3(se::ceil_div(G, kThreads), kColChunks), dim3(kThreads), 0, st,
                         (const TY*)x, L, R, G, sl, sr, (float*)ws);
      SE_LAUNCH_CHECK();
      hipLaunchKernelGGL(bias_col_final_kernel<TY>, dim3(se::ceil_div(G, kThreads)), dim3(kThreads), 0, st,
                         (const float*)ws, G, (TY*)out);
    })
  } else {
    SE_DT_SWITCH(dtype, {
      hipLaunchKernelGGL(bias_row_kernel<TY>, dim3(G), dim3(kThreads), 0, st, (const TY*)x, L, R, sl, sr, sg,
                         (TY*)out);
    })
  }
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_complex_lstm_combine_fwd(const float* h, long long h_lstm_stride, int B, int T, int H, void* out,
                                           long long out_batch_stride, long long out_row_stride,
                                           long long out_feature_stride, int dtype, void* stream) {
  if (!h || !out || B <= 0 || T <= 0 || H <= 0 || h_lstm_stride < 2LL * B * T * H) return SE_E_ARG;
  const long long total = (long long)B * T * 2 * H;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(clstm_combine_fwd_kernel<TY>, dim3(grid_of(total, 4)), dim3(kThreads), 0,
                       se::as_stream(stream), h, h_lstm_stride, B, T, H, (TY*)out, out_batch_stride, out_row_stride,
                       out_feature_stride);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_complex_lstm_combine_bwd(const void* gout, long long g_batch_stride, long long g_row_stride,
                                           long long g_feature_stride, int B, int T, int H, int dtype, float* dh,
                                           long long dh_lstm_stride, void* stream) {
  if (!gout || !dh || B <= 0 || T <= 0 || H <= 0 || dh_lstm_stride < 2LL * B * T * H) return SE_E_ARG;
  const long long total = (long long)B * T * H;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(clstm_combine_bwd_kernel<TY>, dim3(grid_of(total, 4)), dim3(kThreads), 0,
                       se::as_stream(stream), (const TY*)gout, g_batch_stride, g_row_stride, g_feature_stride, B, T, H, dh,
                       dh_lstm_stride);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_carn_mask_fwd(const void* m, long long m_batch_stride, const void* spec, int B, int half, int T,
                                int dtype, void* est, void* stream) {
  if (!m || !spec || !est || B <= 0 || half <= 0 || T <= 0 || B > 65535) return SE_E_ARG;
  const dim3 grid(grid_of((long long)half * T, 4) > 4096 ? 4096 : grid_of((long long)half * T, 4), B);
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(carn_mask_fwd_kernel<TY>, grid, dim3(kThreads), 0, se::as_stream(stream), (const TY*)m,
                       m_batch_stride, (const TY*)spec, half, T, (TY*)est);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_carn_mask_bwd(const void* gest, const void* m, long long m_batch_stride, const void* spec, int B,
                                int half, int T, int dtype, void* dm, void* dspec, void* stream) {
  if (!gest || !m || !spec || !dm || B <= 0 || half <= 0 || T <= 0 || B > 65535) return SE_E_ARG;
  const dim3 grid(grid_of((long long)half * T, 4) > 4096 ? 4096 : grid_of((long long)half * T, 4), B);
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(carn_mask_bwd_kernel<TY>, grid, dim3(kThreads), 0, se::as_stream(stream), (const TY*)gest,
                       (const TY*)m, m_batch_stride, (const TY*)spec, half, T, (TY*)dm, (TY*)dspec);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_add_sigmoid_fwd(const void* a, const void* b, void* y, long long n, int dtype, void* stream) {
  if (!a || !b || !y || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(add_sigmoid_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)a, (const TY*)b, (TY*)y, n);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_sigmoid_fwd(const void* x, void* y, long long n, int dtype, void* stream) {
  if (!x || !y || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(sigmoid_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)x, (TY*)y, n);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_sigmoid_bwd(const void* g, const void* y, void* dz, long long n, int dtype, void* stream) {
  if (!g || !y || !dz || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(sigmoid_bwd_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)g, (const TY*)y, (TY*)dz, n);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_gate_cat_fwd(const void* c, const void* skip, void* out, int B, int C, long long HW, int dtype,
                               void* stream) {
  if (!c || !skip || !out || B <= 0 || C <= 0 || HW <= 0 || B > 65535) return SE_E_ARG;
  const long long CHW = (long long)C * HW;
  const dim3 grid(grid_of(CHW, 4) > 4096 ? 4096 : grid_of(CHW, 4), B);
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(gate_cat_fwd_kernel<TY>, grid, dim3(kThreads), 0, se::as_stream(stream), (const TY*)c,
                       (const TY*)skip, (TY*)out, CHW);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_gate_cat_bwd(const void* gout, const void* c, const void* skip, void* dc, void* dskip, int B, int C,
                               long long HW, int dtype, void* stream) {
  if (!gout || !c || !skip || !dc || !dskip || B <= 0 || C <= 0 || HW <= 0 || B > 65535) return SE_E_ARG;
  const long long CHW = (long long)C * HW;
  const dim3 grid(grid_of(CHW, 4) > 4096 ? 4096 : grid_of(CHW, 4), B);
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(gate_cat_bwd_kernel<TY>, grid, dim3(kThreads), 0, se::as_stream(stream), (const TY*)gout,
                       (const TY*)c, (const TY*)skip, (TY*)dc, (TY*)dskip, CHW);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_glu_fwd(const void* a, const void* b, void* y, long long n, int dtype, void* stream) {
  if (!a || !b || !y || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(glu_fwd_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)a, (const TY*)b, (TY*)y, n);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_glu_bwd(const void* g, const void* a, const void* b, void* da, void* db, long long n, int dtype,
                          void* stream) {
  if (!g || !a || !b || !da || !db || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(glu_bwd_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)g, (const TY*)a, (const TY*)b, (TY*)da, (TY*)db, n);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_clamp_fwd(const void* x, void* y, long long n, float lo, float hi, int dtype, void* stream) {
  if (!x || !y || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(clamp_fwd_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)x, (TY*)y, n, lo, hi);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_clamp_bwd(const void* g, const void* x, void* dx, long long n, float lo, float hi, int dtype,
                            void* stream) {
  if (!g || !x || !dx || n < 0) return SE_E_ARG;
  if (n == 0) return SE_OK;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(clamp_bwd_kernel<TY>, dim3(grid_of(n, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)g, (const TY*)x, (TY*)dx, n, lo, hi);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_chunk_split(const void* x, long long L, int n, int chunk, int hop, int dtype, void* out,
                              void* stream) {
  if (!x || !out || L <= 0 || n <= 0 || chunk <= 0 || hop <= 0 || hop > chunk) return SE_E_ARG;
  const long long total = (long long)n * chunk;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(chunk_split_kernel<TY>, dim3(grid_of(total, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)x, L, chunk, hop, (TY*)out, total);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_chunk_overlap_add(const void* y, int n, int width, int chunk, int overlap, long long length,
                                    int dtype, void* out, void* stream) {
  if (!y || !out || n <= 0 || width <= 0 || chunk <= 0 || overlap < 0 || overlap >= chunk || length <= 0 ||
      length > (long long)(chunk - overlap) * (n - 1) + chunk)
    return SE_E_ARG;
  SE_DT_SWITCH(dtype, {
    hipLaunchKernelGGL(chunk_ola_kernel<TY>, dim3(grid_of(length, 4)), dim3(kThreads), 0, se::as_stream(stream),
                       (const TY*)y, n, width, chunk, overlap, length, (TY*)out);
  })
  SE_LAUNCH_CHECK();
  return SE_OK;
}
