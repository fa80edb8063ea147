// ComplexBatchNorm2d (complex_nn.py:148-329) + fused activation.
//
// Reference cost: ~40 ATen launches per call and >= 4 reads of x
// (SURVEY.md §3.4). Here a training forward is 3 launches and 2 reads of x:
//   cbn_moments_kernel  : one pass, 5 fp64 moments per complex channel
//   cbn_finalize_kernel : mean, covariance, running-stat lerp, the closed
//                         2x2 inverse square root (:288-297), Z = W U
//   cbn_apply_kernel    : y = act(Z (x - M) + B)
// and a training backward is 3 launches reading (gy, x) twice: the activation
// derivative comes from the sign of the pre-activation z = Z (x - M) + B,
// recomputed from x with the forward's own expression, so y is never read
// (2 of the 7 backward passes over the activation of the old design).
// All kernels stream the channel planes contiguously (HBM-bound).
//
// Scale sources of the SE_MATH_F16X3 conv GEMMs (se_conv2d_desc.x_amax /
// dy_amax): the moments passes also keep per-channel extrema (forward: min and
// max of x; backward: max |g|), and the 1-block finalize kernels turn them into
// an upper bound of max |y| (forward) or max |dx| (backward) over the whole
// tensor, e.g. |y_r| <= |Zrr| max|x_r - Mr| + |Zri| max|x_i - Mi| + |Br| (the
// activations never increase a magnitude). No extra pass, no atomics; the bound
// is within a small factor of the true maximum, which the scaled split-fp16
// GEMMs absorb without loss.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int kThreads = 256;
// SE_CBN_APPLY_FIN: the backward finalize in the apply pass's prologue (cbn_bwd_apply_fin_kernel);
// SE_CBN_APPLY_FIN_PR: also with the one-weight PReLU (round 6, variant builds: its prologue
// finalize re-read per apply workgroup cost more than the two launches it saves, DCCRN bf16
// train 1402 / 1406 vs 1410 / 1410 utt/s, profiles/ab/r6_cbn_prelu_fold_ab.log)
#ifndef SE_CBN_APPLY_FIN_PR
#define SE_CBN_APPLY_FIN_PR 0
#endif
#ifndef SE_CBN_APPLY_FIN
#define SE_CBN_APPLY_FIN 1
#endif
constexpr int kSeg = 8192;   // elements of one (b, c) plane per reduction row
constexpr int kSave = 20;    // floats of per-channel state (SE_CBN_SAVE_FLOATS)
// save layout (S_DR / S_DI: max |x_r - Mr|, max |x_i - Mi| of the training batch)
enum { S_MR = 0, S_MI, S_VRR, S_VRI, S_VII, S_URR, S_URI, S_UII,
       S_ZRR, S_ZRI, S_ZIR, S_ZII, S_BR, S_BI, S_S, S_T, S_DR, S_DI, S_PAD0, S_PAD1 };
static_assert(kSave == SE_CBN_SAVE_FLOATS, "save layout");

// block-wide max of v (all threads call); thread 0 gets the result
__device__ __forceinline__ float block_max(float v) {
  __shared__ float red[kThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < (int)(blockDim.x + 63) / 64; ++w) v = fmaxf(v, red[w]);
  return v;
}

// Storage types (SE_DTYPE_*): the activations, and in a bf16 / fp16 model (the
// reference's model.to(bfloat16) / .half()) the module's parameters and running
// statistics too, are T in memory; all arithmetic is fp32 / fp64, loads convert up
// and stores round to nearest even. The per-channel state (save, coef) stays fp32.
struct Ptr5 { const void* p[5]; };
struct MPtr5 { void* p[5]; };
template <typename T> __device__ __forceinline__ float ldv(const void* p, long long i) {
  return (float)static_cast<const T*>(p)[i];
}
template <typename T> __device__ __forceinline__ void stv(void* p, long long i, float v) {
  static_cast<T*>(p)[i] = (T)v;
}
// 4 consecutive elements <-> f32x4 (16-B fp32 / 8-B bf16, fp16 accesses)
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <typename T> __device__ __forceinline__ f32x4v ld4(const T* p) {
  typedef T T4 __attribute__((ext_vector_type(4)));
  return __builtin_convertvector(*reinterpret_cast<const T4*>(p), f32x4v);
}
template <typename T> __device__ __forceinline__ void st4(T* p, f32x4v v) {
  typedef T T4 __attribute__((ext_vector_type(4)));
  *reinterpret_cast<T4*>(p) = __builtin_convertvector(v, T4);
}

template <int NS>
__device__ __forceinline__ void block_reduce_store(double (&v)[NS], double* out) {
  __shared__ double red[kThreads / 64][NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) v[k] = se::wave_sum(v[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < NS; ++k) red[threadIdx.x >> 6][k] = v[k];
  __syncthreads();
  if (threadIdx.x < NS) {
    double s = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += red[w][threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// act 0 none, 1 LeakyReLU(slope), 2 ReLU. Branch-free in the element: act and slope
// are uniform, so the negative-side factor is a scalar select hoisted out of the loops
// and an element costs one compare + select (a branch on act per element splits every
// loop body into scalar-branch blocks).
__device__ __forceinline__ float act_neg(int act, float slope) {
  return act == 1 ? slope : (act == 2 ? 0.f : 1.f);
}
__device__ __forceinline__ float act_grad(float z, int act, float slope) {
  return z > 0.f ? 1.f : act_neg(act, slope);
}
__device__ __forceinline__ float act_fwd(float z, int act, float slope) {
  return z > 0.f ? z : (act == 2 ? 0.f : z * act_neg(act, slope));
}

// grid (Cc, P). Row r = (b, segment) of channel c; rows strided over P.
// ext[(c * P + p) * 4 + {0..3}] = max x_r, -min x_r, max x_i, -min x_i
template <typename T>
__global__ void __launch_bounds__(kThreads)
cbn_moments_kernel(const T* __restrict__ x, int B, int C, int HW, int P, double* part, float* ext,
                   float* y_amax) {
  const int Cc = C / 2, c = blockIdx.x, p = blockIdx.y;
  if (y_amax && c == 0 && p == 0 && threadIdx.x == 0) *y_amax = 0.f;   // the finalize blocks atomicMax into it
  const int nseg = (HW + kSeg - 1) / kSeg;
  double v[5] = {0, 0, 0, 0, 0};
  float e[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int row = p; row < B * nseg; row += P) {
    const int b = row / nseg, sg = row - b * nseg;
    const T* xr = x + ((long long)b * C + c) * HW;
    const T* xi = x + ((long long)b * C + Cc + c) * HW;
    const int i1 = min(HW, (sg + 1) * kSeg);
    auto body = [&](float fr, float fm) __attribute__((always_inline)) {
      e[0] = fmaxf(e[0], fr); e[1] = fmaxf(e[1], -fr); e[2] = fmaxf(e[2], fm); e[3] = fmaxf(e[3], -fm);
      const double r = fr, m = fm;
      v[0] += r; v[1] += m; v[2] += r * r; v[3] += r * m; v[4] += m * m;
    };
    int i = sg * kSeg + threadIdx.x;
    constexpr int U = 4;   // loads of four positions in flight; the sums keep their order
    for (; i + (U - 1) * kThreads < i1; i += U * kThreads) {
      float fr[U], fm[U];
#pragma unroll
      for (int u = 0; u < U; ++u) { fr[u] = (float)xr[i + u * kThreads]; fm[u] = (float)xi[i + u * kThreads]; }
#pragma unroll
      for (int u = 0; u < U; ++u) body(fr[u], fm[u]);
    }
    for (; i < i1; i += kThreads) body((float)xr[i], (float)xi[i]);
  }
  block_reduce_store<5>(v, part + ((long long)c * P + p) * 5);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    __syncthreads();
    const float m = block_max(e[k]);
    if (threadIdx.x == 0) ext[((long long)c * P + p) * 4 + k] = m;
  }
}

// One wave per channel (kFinWaves channels per block): the lanes add the P
// partial rows in parallel; lane 0 does the channel's closed-form math. The
// bound of max |y| goes to *y_amax by atomicMax (zeroed by the moments pass);
// num_batches_tracked is incremented by the apply pass, after every block has
// read it here.
constexpr int kFinWaves = 4;
template <typename T>
__global__ void __launch_bounds__(64 * kFinWaves)
cbn_finalize_kernel(const double* part, const float* ext, int P, double count, int Cc,
                    Ptr5 params, int affine, MPtr5 running, int has_running,
                    const int64_t* nbt, float* save, int training, float eps,
                    float momentum, float* y_amax) {
  float factor = 0.f;
  if (training && has_running) {
    factor = momentum >= 0.f ? momentum : (float)(1.0 / (double)(nbt ? (*nbt + 1) : 1));
  }
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (c >= Cc) return;
  double s[5] = {0, 0, 0, 0, 0};
  float xmax_r = -INFINITY, xmin_r = -INFINITY, xmax_i = -INFINITY, xmin_i = -INFINITY;
  if (training) {
    for (int p = lane; p < P; p += 64) {
#pragma unroll
      for (int k = 0; k < 5; ++k) s[k] += part[((long long)c * P + p) * 5 + k];
      const float* q = ext + ((long long)c * P + p) * 4;
      xmax_r = fmaxf(xmax_r, q[0]); xmin_r = fmaxf(xmin_r, q[1]);
      xmax_i = fmaxf(xmax_i, q[2]); xmin_i = fmaxf(xmin_i, q[3]);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) s[k] = se::wave_sum(s[k]);
    xmax_r = se::wave_max(xmax_r); xmin_r = se::wave_max(xmin_r);
    xmax_i = se::wave_max(xmax_i); xmin_i = se::wave_max(xmin_i);
  }
  if (lane != 0) return;
  {
    double mr, mi, vrr, vri, vii;
    if (training) {
      mr = s[0] / count; mi = s[1] / count;
      vrr = s[2] / count - mr * mr;
      vri = s[3] / count - mr * mi;
      vii = s[4] / count - mi * mi;
      if (has_running) {  // lerp_ in fp32 like the reference (:250-251, :272-274)
        const float nv[5] = {(float)mr, (float)mi, (float)vrr, (float)vri, (float)vii};
        for (int k = 0; k < 5; ++k) {
          const float r = ldv<T>(running.p[k], c);
          stv<T>(running.p[k], c, r + factor * (nv[k] - r));
        }
      }
    } else {
      mr = ldv<T>(running.p[0], c); mi = ldv<T>(running.p[1], c);
      vrr = ldv<T>(running.p[2], c); vri = ldv<T>(running.p[3], c); vii = ldv<T>(running.p[4], c);
    }
    vrr += eps; vii += eps;
    const double s = sqrt(vrr * vii - vri * vri);
    const double t = sqrt(vrr + vii + 2.0 * s);
    const double r = 1.0 / (s * t);
    const double urr = (s + vii) * r, uii = (s + vrr) * r, uri = -vri * r;
    double zrr = urr, zri = uri, zir = uri, zii = uii, br = 0, bi = 0;
    if (affine) {
      const double wrr = ldv<T>(params.p[0], c), wri = ldv<T>(params.p[1], c), wii = ldv<T>(params.p[2], c);
      zrr = wrr * urr + wri * uri;
      zri = wrr * uri + wri * uii;
      zir = wri * urr + wii * uri;
      zii = wri * uri + wii * uii;
      br = ldv<T>(params.p[3], c); bi = ldv<T>(params.p[4], c);
    }
    float* o = save + (long long)c * kSave;
    o[S_MR] = (float)mr; o[S_MI] = (float)mi;
    o[S_VRR] = (float)vrr; o[S_VRI] = (float)vri; o[S_VII] = (float)vii;
    o[S_URR] = (float)urr; o[S_URI] = (float)uri; o[S_UII] = (float)uii;
    o[S_ZRR] = (float)zrr; o[S_ZRI] = (float)zri; o[S_ZIR] = (float)zir; o[S_ZII] = (float)zii;
    o[S_BR] = (float)br; o[S_BI] = (float)bi; o[S_S] = (float)s; o[S_T] = (float)t;
    float dr = INFINITY, di = INFINITY;   // eval: the batch extrema are unknown
    if (training) {
      // max |x - M| (xmin_* hold -min); rounded up so the bound stays a bound
      dr = fmaxf(xmax_r - (float)mr, xmin_r + (float)mr) * 1.0001f;
      di = fmaxf(xmax_i - (float)mi, xmin_i + (float)mi) * 1.0001f;
      const float yr = fabsf((float)zrr) * dr + fabsf((float)zri) * di + fabsf((float)br);
      const float yi = fabsf((float)zir) * dr + fabsf((float)zii) * di + fabsf((float)bi);
      if (y_amax) atomicMax(reinterpret_cast<unsigned*>(y_amax), __float_as_uint(fmaxf(yr, yi) * 1.0001f));
    }
    o[S_DR] = dr; o[S_DI] = di; o[S_PAD0] = o[S_PAD1] = 0.f;
  }
}

// grid (ceil(HW / (kThreads*4)), Cc, B). pw != NULL: nn.PReLU() (one weight,
// dccrn.py:21,45) as LeakyReLU with the slope read from the device parameter.
template <typename T>
__global__ void __launch_bounds__(kThreads)
cbn_apply_kernel(const T* __restrict__ x, T* __restrict__ y, int C, int HW,
                 const float* __restrict__ save, int act, float slope, int64_t* nbt, const T* pw) {
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  if (pw) slope = (float)pw[0];
  if (nbt && blockIdx.x == 0 && c == 0 && b == 0 && threadIdx.x == 0) *nbt += 1;   // num_batches_tracked
  const float* s = save + c * kSave;
  const float mr = s[S_MR], mi = s[S_MI], zrr = s[S_ZRR], zri = s[S_ZRI];
  const float zir = s[S_ZIR], zii = s[S_ZII], br = s[S_BR], bi = s[S_BI];
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int base = blockIdx.x * kThreads * 4 + threadIdx.x;
  float fxr[4], fxi[4];   // the four positions' loads first (clamped index), stores guarded
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = min(base + u * kThreads, HW - 1);
    fxr[u] = (float)x[offr + j];
    fxi[u] = (float)x[offi + j];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = base + u * kThreads;
    if (i < HW) {
      const float xr = fxr[u] - mr, xi = fxi[u] - mi;
      const float yr = act_fwd(zrr * xr + zri * xi + br, act, slope);
      const float yi = act_fwd(zir * xr + zii * xi + bi, act, slope);
      y[offr + i] = (T)yr;
      y[offi + i] = (T)yi;
    }
  }
}

// cbn_apply_kernel with 16-B accesses (HW % 4 == 0: every plane starts 16-B
// aligned): one float4 of the real and one of the imaginary plane per thread.
// grid (ceil(HW / (kThreads*4)), Cc, B)
template <typename T>
__global__ void __launch_bounds__(kThreads)
cbn_apply4_kernel(const T* __restrict__ x, T* __restrict__ y, int C, int HW,
                  const float* __restrict__ save, int act, float slope, int64_t* nbt, const T* pw) {
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  if (pw) slope = (float)pw[0];
  if (nbt && blockIdx.x == 0 && c == 0 && b == 0 && threadIdx.x == 0) *nbt += 1;   // num_batches_tracked
  const float* s = save + c * kSave;
  const float mr = s[S_MR], mi = s[S_MI], zrr = s[S_ZRR], zri = s[S_ZRI];
  const float zir = s[S_ZIR], zii = s[S_ZII], br = s[S_BR], bi = s[S_BI];
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int i = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (i >= HW) return;
  const f32x4v xr4 = ld4(x + offr + i);
  const f32x4v xi4 = ld4(x + offi + i);
  f32x4v yr4, yi4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float xr = xr4[u] - mr, xi = xi4[u] - mi;
    yr4[u] = act_fwd(zrr * xr + zri * xi + br, act, slope);
    yi4[u] = act_fwd(zir * xr + zii * xi + bi, act, slope);
  }
  st4(y + offr + i, yr4);
  st4(y + offi + i, yi4);
}

// Output head of FRCRN (frcrn.py:115, 140-144): final_conv = nn.Conv2d(C, 2, (1, 2),
// bias=False) applied to y = act(CBN(x)) of the last decoder block. Nothing else
// reads that y, so it is never written: the forward computes the head straight
// from x (cbn_head_apply_kernel), and the backward forms dL/dy from the head's
// gradient g [B, 2, H, W-1] on the fly,
//   gy_c(h, t) = sum_o w[o, c, 0] g_o(h, t) + w[o, c, 1] g_o(h, t - 1)   (zero off the grid),
// inside both backward passes, while the moments pass also sums the head's
// weight gradient dw[o, c, k] = sum g_o(h, t) y_c(h, t + k) from y recomputed.
constexpr int kHeadNO = 2;   // head output channels
constexpr int kHeadKW = 2;   // head kernel width (time taps)
constexpr int kHeadNS = 8;   // extra moments per complex channel: 2 parts x NO x KW
struct HeadArgs {
  const float* g;   // [B, NO, H, W - 1]
  const float* w;   // [NO, C, 1, KW]
  int W;            // input time width
};

// g_o at (b, row, t) and (b, row, t - 1) for both outputs, zero off the grid
struct HeadG { float g0[kHeadNO], g1[kHeadNO]; };
__device__ __forceinline__ HeadG head_g(const HeadArgs& h, int b, int H, int row, int t) {
  HeadG r;
  const int W1 = h.W - 1;
#pragma unroll
  for (int o = 0; o < kHeadNO; ++o) {
    const float* go = h.g + (((long long)b * kHeadNO + o) * H + row) * W1;
    r.g0[o] = t < W1 ? go[t] : 0.f;
    r.g1[o] = t >= 1 ? go[t - 1] : 0.f;
  }
  return r;
}

// dL/dy of real channel ch from the head gradient (wc: w[o, ch, k] at o * C * KW + k)
__device__ __forceinline__ float head_gy(const HeadG& g, const float* wc, int C) {
  float s = 0.f;
#pragma unroll
  for (int o = 0; o < kHeadNO; ++o) s += wc[o * C * kHeadKW] * g.g0[o] + wc[o * C * kHeadKW + 1] * g.g1[o];
  return s;
}

// coef layout per channel (16 floats): ZTrr ZTri ZTir ZTii gbr gbi Grr Gri Gii Mr Mi Br Bi pad
constexpr int kCoef = 16;

// SRC 3 (se_cbn_bwd_ccbam): dL/dy = gy + the input gradient of the CCBAM gate that reads
// the forked output (FRCRN's encoder skip, frcrn.py:70-75 + ccbam.py:95-106), formed on the
// fly from the gate's parts instead of being written by ccbam.hip's bwd_dx_kernel and read
// back: at (b, channel ch = h Ch + cc, position i)
//   gy2 = (g + dP[b, 2h, i] / Ch + [idx[b, h, i] == cc] dP[b, 2h + 1, i]) ca[b, ch]
//         + dmean[b, ch] / HW + [amax[b, ch] == i] dmax[b, ch]
// (bwd_dx_kernel's expression, term for term). fp32 only.
struct CcbamDx {
  const float* g;       // [B, C, HW] the gate's output gradient
  const float* dP;      // [B, 4, HW] pooled-map gradient (avg_re, max_re, avg_im, max_im)
  const short* idx;     // [B, 2, HW] channel argmax per half
  const float* ca;      // [B, C] channel gate
  const float* dmean;   // [B, C]
  const float* dmax;    // [B, C]
  const int* amax;      // [B, C] HW argmax
};
struct CcbRow { float ca, mean, mx; int am; };   // one (b, channel) plane's constants
__device__ __forceinline__ CcbRow ccb_row(const CcbamDx& cd, long long bc, float invhw) {
  return CcbRow{cd.ca[bc], cd.dmean[bc] * invhw, cd.dmax[bc], cd.amax[bc]};
}
// gy2 of plane h at position i, given the position's pooled-map terms
__device__ __forceinline__ float ccb_dx(float g, float pa, float pm, int pi, int cc, const CcbRow& r, int i) {
  const float gx = g + pa + (pi == cc ? pm : 0.f);
  return gx * r.ca + r.mean + (r.am == i ? r.mx : 0.f);
}

// One wave per channel, as cbn_finalize_kernel; the bound of max |dx| goes to
// *dx_amax by atomicMax (zeroed by the backward moments pass).
// HEAD: part holds the head's 8 weight-grad sums after the 6 moments (stride
// 6 + kHeadNS); they are added in the same fixed order and written to dwh.
// PR: the 7th sum (the PReLU weight's gradient, per channel) goes to pw_part[c]
// o: the channel's kCoef floats; side: also write the parameter gradients, the head
// weight gradient, the PReLU partial and the dx bound (once per channel)
template <bool HEAD, typename T = float, bool PR = false>
__device__ __forceinline__ void bwd_finalize_wave(int c, int lane, const double* part, const float* ext, int P,
                                                  double count, int Cc, const float* save, const Ptr5& params,
                                                  int affine, const MPtr5& dparams, int has_dparams, int training,
                                                  float* o, float* dx_amax, float* dwh, double* pw_part,
                                                  bool side) {
  constexpr int NS = HEAD ? 6 + kHeadNS : (PR ? 7 : 6);
  double sm[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) sm[k] = 0;
  float gmr = 0.f, gmi = 0.f;
  for (int p = lane; p < P; p += 64) {
#pragma unroll
    for (int k = 0; k < NS; ++k) sm[k] += part[((long long)c * P + p) * NS + k];
    gmr = fmaxf(gmr, ext[((long long)c * P + p) * 2 + 0]);
    gmi = fmaxf(gmi, ext[((long long)c * P + p) * 2 + 1]);
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) sm[k] = se::wave_sum(sm[k]);
  gmr = se::wave_max(gmr);
  gmi = se::wave_max(gmi);
  if (lane != 0) return;
  if constexpr (PR) {
    if (side) pw_part[c] = sm[NS - 1];
  }
  if (HEAD && side) {   // dw[o, ch, k] at (o * C + ch) * KW + k, C = 2 Cc
    const int C = 2 * Cc;
#pragma unroll
    for (int o = 0; o < kHeadNO; ++o)
#pragma unroll
      for (int k = 0; k < kHeadKW; ++k) {
        dwh[((long long)o * C + c) * kHeadKW + k] = (float)sm[6 + 2 * o + k];
        dwh[((long long)o * C + Cc + c) * kHeadKW + k] = (float)sm[10 + 2 * o + k];
      }
  }
  {
    const float* s = save + (long long)c * kSave;
    const double urr = s[S_URR], uri = s[S_URI], uii = s[S_UII];
    const double vrr = s[S_VRR], vri = s[S_VRI], vii = s[S_VII];
    const double ss = s[S_S], tt = s[S_T];
    // dZ = sum g xt^T
    const double dz00 = sm[2], dz01 = sm[3], dz10 = sm[4], dz11 = sm[5];
    double wrr = 1, wri = 0, wii = 1;
    if (affine) { wrr = ldv<T>(params.p[0], c); wri = ldv<T>(params.p[1], c); wii = ldv<T>(params.p[2], c); }
    double gurr, guri, guii;
    if (affine) {
      // dW = dZ U (U symmetric); W symmetric -> Wri collects both off-diagonals
      const double dw00 = dz00 * urr + dz01 * uri, dw01 = dz00 * uri + dz01 * uii;
      const double dw10 = dz10 * urr + dz11 * uri, dw11 = dz10 * uri + dz11 * uii;
      if (has_dparams && side) {
        stv<T>(dparams.p[0], c, (float)dw00);
        stv<T>(dparams.p[1], c, (float)(dw01 + dw10));
        stv<T>(dparams.p[2], c, (float)dw11);
        stv<T>(dparams.p[3], c, (float)sm[0]);
        stv<T>(dparams.p[4], c, (float)sm[1]);
      }
      // dU = W^T dZ = W dZ
      gurr = wrr * dz00 + wri * dz10;
      guii = wri * dz01 + wii * dz11;
      guri = (wrr * dz01 + wri * dz11) + (wri * dz00 + wii * dz10);
    } else {
      gurr = dz00; guii = dz11; guri = dz01 + dz10;
    }
    const double zrr = s[S_ZRR], zri = s[S_ZRI], zir = s[S_ZIR], zii = s[S_ZII];
    double gbr = 0, gbi = 0, grr = 0, gri = 0, gii = 0;
    if (training) {
      // back through U(Vrr, Vri, Vii) = closed form with s = sqrt(det), t = sqrt(tr + 2s)
      const double r = 1.0 / (ss * tt);
      const double g_r = gurr * (ss + vii) + guii * (ss + vrr) - guri * vri;
      const double g_t = -g_r * r / tt;
      const double g_s = (gurr + guii) * r - g_r * r / ss + g_t / tt;
      const double g_tau = g_t / (2.0 * tt);
      const double g_del = g_s / (2.0 * ss);
      const double gvrr = guii * r + g_tau + g_del * vii;
      const double gvii = gurr * r + g_tau + g_del * vrr;
      const double gvri = -guri * r - 2.0 * vri * g_del;
      grr = 2.0 * gvrr / count; gri = gvri / count; gii = 2.0 * gvii / count;
      gbr = sm[0] / count; gbi = sm[1] / count;
    }
    o[0] = (float)zrr; o[1] = (float)zir;   // dxr = Zrr g_r + Zir g_i
    o[2] = (float)zri; o[3] = (float)zii;   // dxi = Zri g_r + Zii g_i
    o[4] = (float)gbr; o[5] = (float)gbi;
    o[6] = (float)grr; o[7] = (float)gri; o[8] = (float)gii;
    o[9] = s[S_MR]; o[10] = s[S_MI]; o[11] = s[S_BR]; o[12] = s[S_BI];
    o[13] = o[14] = o[15] = 0.f;
    if (side && training && dx_amax) {   // dx = Z^T (g - gb) + Gamma (x - M), bounded term by term
      const float gr = gmr + fabsf(o[4]);
      const float gi = gmi + fabsf(o[5]);
      const float dr = s[S_DR], di = s[S_DI];
      const float br = fabsf(o[0]) * gr + fabsf(o[1]) * gi + fabsf(o[6]) * dr + fabsf(o[7]) * di;
      const float bi = fabsf(o[2]) * gr + fabsf(o[3]) * gi + fabsf(o[7]) * dr + fabsf(o[8]) * di;
      atomicMax(reinterpret_cast<unsigned*>(dx_amax), __float_as_uint(fmaxf(br, bi) * 1.0001f));
    }
  }
}

template <bool HEAD, typename T = float, bool PR = false>
__global__ void __launch_bounds__(64 * kFinWaves)
cbn_bwd_finalize_kernel(const double* part, const float* ext, int P, double count, int Cc,
                        const float* save, Ptr5 params, int affine,
                        MPtr5 dparams, int has_dparams, int training,
                        float* coef, float* dx_amax, float* dwh, double* pw_part) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (c >= Cc) return;
  bwd_finalize_wave<HEAD, T, PR>(c, lane, part, ext, P, count, Cc, save, params, affine, dparams, has_dparams,
                                 training, coef + (long long)c * kCoef, dx_amax, dwh, pw_part, true);
}

// The backward apply (SRC 0 / 1, cbn_bwd_apply(4)_kernel's arithmetic) with the finalize in
// its prologue: a workgroup per (channel, item) runs the channel's finalize into LDS (wave
// 0; the parameter gradients and the dx bound from the item-0 workgroups) and then streams
// the item's two planes. One main-stream launch fewer per CBN backward: beside the
// side-stream weight-grads the 16-workgroup finalize launch waited 60-310 us for CU slots
// (profiles/r4_main_stream_kernels.txt). V4: 16-B accesses (HW % 4 == 0). grid (Cc, B)
// PR: the one-weight nn.PReLU (DCCRN): the slope is read from pw, the channel's writer
// workgroup stores its PReLU-gradient sum to pw_part[c], and the last of the Cc writers
// (a device-scope count, zeroed by the moments pass) adds them in channel order into dpw
// (prelu_grad_finish_kernel's sum): no separate finalize / finish launches.
template <int SRC, typename T, bool V4, bool PR = false>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply_fin_kernel(const T* __restrict__ gy, const T* __restrict__ gy2, const T* __restrict__ x,
                         T* __restrict__ dx, int C, int HW, int seg_len, int act, float slope,
                         const double* part, const float* ext, int P, double count, const float* save, Ptr5 params,
                         int affine, MPtr5 dparams, int has_dparams, int training, float* dx_amax, CcbamDx cd,
                         const T* pw, T* dpw, double* pw_part, unsigned* pw_cnt) {
  static_assert(SRC == 0 || SRC == 1 || SRC == 3, "gy, gy + gy2, or gy + the CCBAM gate's input gradient");
  static_assert(SRC != 3 || sizeof(T) == 4, "the CCBAM path is fp32");
  static_assert(!PR || SRC != 3, "no PReLU on the CCBAM path");
  __shared__ float k[kCoef];
  const int Cc = C / 2, c = blockIdx.x, b = blockIdx.y;
  const int hw0 = blockIdx.z * seg_len, hw1 = min(HW, hw0 + seg_len);   // this workgroup's segment
  if constexpr (PR) slope = (float)pw[0];
  const bool writer = b == 0 && blockIdx.z == 0;
  if (threadIdx.x < 64)
    bwd_finalize_wave<false, T, PR>(c, threadIdx.x, part, ext, P, count, Cc, save, params, affine, dparams,
                                    has_dparams, training, k, dx_amax, nullptr, pw_part, writer);
  if constexpr (PR) {
    if (writer && threadIdx.x == 0) {
      __threadfence();   // pw_part[c] visible device-wide before the count moves
      if (atomicAdd(pw_cnt, 1u) == (unsigned)(Cc - 1)) {
        __threadfence();
        double sacc = 0.0;
        for (int q = 0; q < Cc; ++q) sacc += __hip_atomic_load(&pw_part[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dpw[0] = (T)(float)sacc;
      }
    }
  }
  __syncthreads();
  const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
  const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
  const float br = k[11], bi = k[12];
  const float neg = act_neg(act, slope);
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  CcbRow rr{}, ri{};
  const float* dPb = nullptr;
  const short* ib = nullptr;
  const float cinv = 1.f / (float)Cc, invhw = 1.f / (float)HW;
  if constexpr (SRC == 3) {
    rr = ccb_row(cd, (long long)b * C + c, invhw);
    ri = ccb_row(cd, (long long)b * C + Cc + c, invhw);
    dPb = cd.dP + (long long)b * 4 * HW;
    ib = cd.idx + (long long)b * 2 * HW;
  }
  auto gate = [&](long long off, int j, int h) __attribute__((always_inline)) -> float {   // SRC 3's gy2
    return ccb_dx(cd.g[off + j], dPb[(2 * h) * HW + j] * cinv, dPb[(2 * h + 1) * HW + j], ib[h * HW + j], c,
                  h ? ri : rr, j);
  };
  auto one = [&](float fxr, float fxi, float fgr, float fgi, float& dr, float& di) __attribute__((always_inline)) {
    const float xr = fxr - mr, xi = fxi - mi;
    const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
    const float gr = (zr > 0.f ? fgr : fgr * neg) - gbr;
    const float gi = (zi > 0.f ? fgi : fgi * neg) - gbi;
    dr = a00 * gr + a01 * gi + grr * xr + gri * xi;
    di = a10 * gr + a11 * gi + gri * xr + gii * xi;
  };
  if constexpr (V4) {
    constexpr int U = 2;   // float4s per plane and tensor in flight
    for (int i0 = hw0 + threadIdx.x * 4; i0 < hw1; i0 += kThreads * 4 * U) {
      f32x4v xr4[U], xi4[U], gr4[U], gi4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * kThreads * 4, HW - 4);   // clamped loads, guarded stores
        xr4[u] = ld4(x + offr + i);
        xi4[u] = ld4(x + offi + i);
        gr4[u] = ld4(gy + offr + i);
        gi4[u] = ld4(gy + offi + i);
        if (SRC == 1) {
          gr4[u] += ld4(gy2 + offr + i);
          gi4[u] += ld4(gy2 + offi + i);
        }
        if constexpr (SRC == 3) {   // the gate's parts as 16-B / 8-B loads
          const f32x4v g0 = ld4(cd.g + offr + i), g1 = ld4(cd.g + offi + i);
          const f32x4v pa0 = ld4(dPb + i), pm0 = ld4(dPb + HW + i);
          const f32x4v pa1 = ld4(dPb + 2 * HW + i), pm1 = ld4(dPb + 3 * HW + i);
          typedef short s16x4v __attribute__((ext_vector_type(4)));
          const s16x4v i0 = *reinterpret_cast<const s16x4v*>(ib + i);
          const s16x4v i1 = *reinterpret_cast<const s16x4v*>(ib + HW + i);
#pragma unroll
          for (int l = 0; l < 4; ++l) {
            gr4[u][l] += ccb_dx(g0[l], pa0[l] * cinv, pm0[l], i0[l], c, rr, i + l);
            gi4[u][l] += ccb_dx(g1[l], pa1[l] * cinv, pm1[l], i1[l], c, ri, i + l);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * kThreads * 4;
        if (i < hw1) {
          f32x4v dr4, di4;
#pragma unroll
          for (int l = 0; l < 4; ++l) {
            float dr, di;
            one(xr4[u][l], xi4[u][l], gr4[u][l], gi4[u][l], dr, di);
            dr4[l] = dr;
            di4[l] = di;
          }
          st4(dx + offr + i, dr4);
          st4(dx + offi + i, di4);
        }
      }
    }
  } else {
    constexpr int U = 4;
    for (int i0 = hw0 + threadIdx.x; i0 < hw1; i0 += kThreads * U) {
      float fxr[U], fxi[U], fgr[U], fgi[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(i0 + u * kThreads, HW - 1);
        fxr[u] = (float)x[offr + j];
        fxi[u] = (float)x[offi + j];
        fgr[u] = SRC == 1 ? (float)gy[offr + j] + (float)gy2[offr + j] : (float)gy[offr + j];
        fgi[u] = SRC == 1 ? (float)gy[offi + j] + (float)gy2[offi + j] : (float)gy[offi + j];
        if constexpr (SRC == 3) {
          fgr[u] += gate(offr, j, 0);
          fgi[u] += gate(offi, j, 1);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * kThreads;
        if (i < hw1) {
          float dr, di;
          one(fxr[u], fxi[u], fgr[u], fgi[u], dr, di);
          dx[offr + i] = (T)dr;
          dx[offi + i] = (T)di;
        }
      }
    }
  }
}


// Backward moments: g = dL/dy * act'(z), xt = x - M, with dL/dy = gy (SRC 0),
// gy + gy2 (SRC 1: a forked output, se_cbn_bwd2, summed on the fly) or formed
// from the head gradient (SRC 2, see HeadArgs; then the head's 8 weight-grad
// sums per complex channel follow the 6 below in part, stride NS).
// sums: gr, gi, gr*xtr, gr*xti, gi*xtr, gi*xti; PR (nn.PReLU, slope from pw): a 7th,
// sum dL/dy * z [z <= 0] over both planes (the PReLU weight's gradient)
template <int SRC, typename T = float, bool PR = false>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_moments_kernel(const T* __restrict__ gy, const T* __restrict__ gy2,
                       const T* __restrict__ x, int B, int C, int HW, int P,
                       const float* __restrict__ save, int act, float slope, double* part, float* ext,
                       float* dx_amax, HeadArgs hd, const T* pw, CcbamDx cd, unsigned* pw_cnt) {
  static_assert(!PR || SRC != 2, "no PReLU on the head path");
  static_assert((SRC != 2 && SRC != 3) || sizeof(T) == 4, "the head and CCBAM paths are fp32");
  constexpr int NS = SRC == 2 ? 6 + kHeadNS : (PR ? 7 : 6);
  if (PR) slope = (float)pw[0];
  const int Cc = C / 2, c = blockIdx.x, p = blockIdx.y;
  if (dx_amax && c == 0 && p == 0 && threadIdx.x == 0) *dx_amax = 0.f;   // the finalize blocks atomicMax into it
  if (pw_cnt && c == 0 && p == 0 && threadIdx.x == 0) *pw_cnt = 0u;      // cbn_bwd_apply_fin_kernel<PR>'s count
  const int nseg = (HW + kSeg - 1) / kSeg;
  const float* sv = save + c * kSave;
  float gmr = 0.f, gmi = 0.f;   // max |g_r|, max |g_i| (the dx bound)
  const float mr = sv[S_MR], mi = sv[S_MI];
  const float zrr = sv[S_ZRR], zri = sv[S_ZRI], zir = sv[S_ZIR], zii = sv[S_ZII], br = sv[S_BR], bi = sv[S_BI];
  double v[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) v[k] = 0;
  const int H = SRC == 2 ? HW / hd.W : 1;
  const float* wcr = SRC == 2 ? hd.w + c * kHeadKW : nullptr;
  const float* wci = SRC == 2 ? hd.w + (Cc + c) * kHeadKW : nullptr;
  for (int row = p; row < B * nseg; row += P) {
    const int b = row / nseg, sg = row - b * nseg;
    const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
    const int i1 = min(HW, (sg + 1) * kSeg);
    int i = sg * kSeg + threadIdx.x;
    int hr = 0, ht = 0;   // (row, t) of i in the head's grid, stepped with i
    if (SRC == 2) { hr = i / hd.W; ht = i - hr * hd.W; }
    auto body = [&](float fxr, float fxi, float dyr, float dyi, const HeadG& hg) __attribute__((always_inline)) {
      const float xr = fxr - mr, xi = fxi - mi;
      const float zr = zrr * xr + zri * xi + br, zi = zir * xr + zii * xi + bi;   // = forward pre-activation
      const float gr = dyr * act_grad(zr, act, slope);
      const float gi = dyi * act_grad(zi, act, slope);
      gmr = fmaxf(gmr, fabsf(gr)); gmi = fmaxf(gmi, fabsf(gi));
      v[0] += gr; v[1] += gi;
      v[2] += (double)gr * xr; v[3] += (double)gr * xi;
      v[4] += (double)gi * xr; v[5] += (double)gi * xi;
      if constexpr (PR) v[NS - 1] += (zr <= 0.f ? (double)dyr * zr : 0.0) + (zi <= 0.f ? (double)dyi * zi : 0.0);
      if (SRC == 2) {
        const double yr = act_fwd(zr, act, slope), yi = act_fwd(zi, act, slope);
#pragma unroll
        for (int o = 0; o < kHeadNO; ++o) {
          v[6 + 2 * o] += hg.g0[o] * yr;      // dw[o, c_r, 0]: g(t) y(t)
          v[7 + 2 * o] += hg.g1[o] * yr;      // dw[o, c_r, 1]: g(t - 1) y(t)
          v[10 + 2 * o] += hg.g0[o] * yi;     // dw[o, c_i, 0]
          v[11 + 2 * o] += hg.g1[o] * yi;     // dw[o, c_i, 1]
        }
      }
    };
    if (SRC == 2) {
      // four positions per iteration, every load issued before the arithmetic
      constexpr int U = 4;
      for (; i + (U - 1) * kThreads < i1; i += U * kThreads) {
        float fr[U], fm[U];
        HeadG hg[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          fr[u] = (float)x[offr + i + u * kThreads];
          fm[u] = (float)x[offi + i + u * kThreads];
          hg[u] = head_g(hd, b, H, hr, ht);
          ht += kThreads;
          while (ht >= hd.W) { ht -= hd.W; ++hr; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) body(fr[u], fm[u], head_gy(hg[u], wcr, C), head_gy(hg[u], wci, C), hg[u]);
      }
      for (; i < i1; i += kThreads) {
        const HeadG hg = head_g(hd, b, H, hr, ht);
        body((float)x[offr + i], (float)x[offi + i], head_gy(hg, wcr, C), head_gy(hg, wci, C), hg);
        ht += kThreads;
        while (ht >= hd.W) { ht -= hd.W; ++hr; }
      }
    } else {
      const HeadG none{};
      // SRC 3: the row's gate constants and pooled-map rows
      CcbRow rr{}, ri{};
      const float* dPb = nullptr;
      const short* ib = nullptr;
      const float inv = 1.f / (float)Cc, invhw = 1.f / (float)HW;
      if constexpr (SRC == 3) {
        rr = ccb_row(cd, (long long)b * C + c, invhw);
        ri = ccb_row(cd, (long long)b * C + Cc + c, invhw);
        dPb = cd.dP + (long long)b * 4 * HW;
        ib = cd.idx + (long long)b * 2 * HW;
      }
      auto dy = [&](long long off, int j, int h) __attribute__((always_inline)) -> float {
        if constexpr (SRC == 1) return (float)gy[off + j] + (float)gy2[off + j];
        if constexpr (SRC == 3)
          return (float)gy[off + j] + ccb_dx(cd.g[off + j], dPb[(2 * h) * HW + j] * inv, dPb[(2 * h + 1) * HW + j],
                                             ib[h * HW + j], c, h ? ri : rr, j);
        return (float)gy[off + j];
      };
      constexpr int U = 4;   // loads of four positions in flight; the sums keep their order
      for (; i + (U - 1) * kThreads < i1; i += U * kThreads) {
        float fr[U], fm[U], dr[U], dm[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = i + u * kThreads;
          fr[u] = (float)x[offr + j];
          fm[u] = (float)x[offi + j];
          dr[u] = dy(offr, j, 0);
          dm[u] = dy(offi, j, 1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) body(fr[u], fm[u], dr[u], dm[u], none);
      }
      for (; i < i1; i += kThreads) body((float)x[offr + i], (float)x[offi + i], dy(offr, i, 0), dy(offi, i, 1), none);
    }
  }
  block_reduce_store<NS>(v, part + ((long long)c * P + p) * NS);
  __syncthreads();
  gmr = block_max(gmr);
  __syncthreads();
  gmi = block_max(gmi);
  if (threadIdx.x == 0) {
    ext[((long long)c * P + p) * 2 + 0] = gmr;
    ext[((long long)c * P + p) * 2 + 1] = gmi;
  }
}


template <int SRC, typename T = float>   // dL/dy source as cbn_bwd_moments_kernel
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply_kernel(const T* __restrict__ gy, const T* __restrict__ gy2,
                     const T* __restrict__ x, T* __restrict__ dx, int C, int HW,
                     const float* __restrict__ coef, int act, float slope, HeadArgs hd, const T* pw) {
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  if (pw) slope = (float)pw[0];
  const float* k = coef + c * kCoef;
  const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
  const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
  const float br = k[11], bi = k[12];
  const int H = SRC == 2 ? HW / hd.W : 1;
  // forward Z = [[a00, a10], [a01, a11]] (coef holds Z^T)
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int base = blockIdx.x * kThreads * 4 + threadIdx.x;
  if constexpr (SRC != 2) {
    // the four positions' loads first (clamped index; the stores stay guarded), so a thread
    // keeps them all in flight instead of one position's latency after another
    float fxr[4], fxi[4], fgr[4], fgi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = min(base + u * kThreads, HW - 1);
      fxr[u] = (float)x[offr + j];
      fxi[u] = (float)x[offi + j];
      fgr[u] = SRC == 1 ? (float)gy[offr + j] + (float)gy2[offr + j] : (float)gy[offr + j];
      fgi[u] = SRC == 1 ? (float)gy[offi + j] + (float)gy2[offi + j] : (float)gy[offi + j];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * kThreads;
      if (i < HW) {
        const float xr = fxr[u] - mr, xi = fxi[u] - mi;
        const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
        const float gr = fgr[u] * act_grad(zr, act, slope) - gbr;
        const float gi = fgi[u] * act_grad(zi, act, slope) - gbi;
        dx[offr + i] = (T)(a00 * gr + a01 * gi + grr * xr + gri * xi);
        dx[offi + i] = (T)(a10 * gr + a11 * gi + gri * xr + gii * xi);
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = base + u * kThreads;
    if (i < HW) {
      const float xr = (float)x[offr + i] - mr, xi = (float)x[offi + i] - mi;
      const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
      float dyr, dyi;
      if (SRC == 2) {
        const int hr = i / hd.W;
        const HeadG hg = head_g(hd, b, H, hr, i - hr * hd.W);
        dyr = head_gy(hg, hd.w + c * kHeadKW, C);
        dyi = head_gy(hg, hd.w + (Cc + c) * kHeadKW, C);
      } else {
        dyr = SRC == 1 ? (float)gy[offr + i] + (float)gy2[offr + i] : (float)gy[offr + i];
        dyi = SRC == 1 ? (float)gy[offi + i] + (float)gy2[offi + i] : (float)gy[offi + i];
      }
      const float gr = dyr * act_grad(zr, act, slope) - gbr;
      const float gi = dyi * act_grad(zi, act, slope) - gbi;
      dx[offr + i] = (T)(a00 * gr + a01 * gi + grr * xr + gri * xi);
      dx[offi + i] = (T)(a10 * gr + a11 * gi + gri * xr + gii * xi);
    }
  }
}

// cbn_bwd_apply_kernel<SRC 0 / 1> with 16-B accesses (HW % 4 == 0)
template <int SRC, typename T = float>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply4_kernel(const T* __restrict__ gy, const T* __restrict__ gy2,
                      const T* __restrict__ x, T* __restrict__ dx, int C, int HW,
                      const float* __restrict__ coef, int act, float slope, const T* pw) {
  static_assert(SRC == 0 || SRC == 1, "gy or gy + gy2");
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  if (pw) slope = (float)pw[0];
  const float* k = coef + c * kCoef;
  const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
  const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
  const float br = k[11], bi = k[12];
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int i = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (i >= HW) return;
  const f32x4v xr4 = ld4(x + offr + i);
  const f32x4v xi4 = ld4(x + offi + i);
  f32x4v gr4 = ld4(gy + offr + i);
  f32x4v gi4 = ld4(gy + offi + i);
  if (SRC == 1) {
    gr4 += ld4(gy2 + offr + i);
    gi4 += ld4(gy2 + offi + i);
  }
  f32x4v dr4, di4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float xr = xr4[u] - mr, xi = xi4[u] - mi;
    const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
    const float gr = gr4[u] * act_grad(zr, act, slope) - gbr;
    const float gi = gi4[u] * act_grad(zi, act, slope) - gbi;
    dr4[u] = a00 * gr + a01 * gi + grr * xr + gri * xi;
    di4[u] = a10 * gr + a11 * gi + gri * xr + gii * xi;
  }
  st4(dx + offr + i, dr4);
  st4(dx + offi + i, di4);
}

// sum over the channels (fixed order, fp64) of the per-channel PReLU weight-grad sums
template <typename T>
__global__ void prelu_grad_finish_kernel(const double* pw_part, int Cc, T* dpw) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int c = 0; c < Cc; ++c) s += pw_part[c];
  dpw[0] = (T)(float)s;
}

// First block's conv weight gradient fused into the backward apply (se_cbn_bwd_first_conv).
// The block is conv -> CBN (+ act) with a conv input x0 that needs no gradient (a
// model's first, data-fed conv: FRCRN's encoder layer 0, frcrn.py:28-34). The apply
// pass computes dL/dy0 = dx at each position anyway; instead of writing it (the
// conv's dy, one activation-sized tensor) for a separate weight-grad GEMM to read
// back, each thread multiplies it into the conv's gathered input taps right away:
//   dWr[c, ci, t] += gr * xr + gi * xi,   dWi[c, ci, t] += gi * xr - gr * xi
// (complex_nn.py:52-65: re = Wr*xr - Wi*xi, im = Wi*xr + Wr*xi), xr / xi the real /
// imaginary input channel ci at tap t of the position (zero outside the grid).
// Exact fp32 products, per-thread sums in position order, a fixed-order block
// reduction; per (channel, batch item) partials summed over the items in fp64 by
// cbn_first_conv_finish_kernel. grid (Cc, B), one workgroup per (channel, item) plane.
struct FirstConv {
  const float* x0;    // [B, 2 cin, Hi, Wi]
  int Hi, Wi, sh, sw, ph, pw, dh, dw;
  float* dwr;         // [Cc, cin, KH, KW]
  float* dwi;
};

template <int SRC, int CIN, int KH, int KW>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply_fc_kernel(const float* __restrict__ gy, const float* __restrict__ gy2,
                        const float* __restrict__ x, int C, int HW, int W, const float* __restrict__ coef,
                        int act, float slope, FirstConv fc, float* __restrict__ wpart) {
  static_assert(SRC == 0 || SRC == 1, "gy or gy + gy2");
  constexpr int NT = CIN * KH * KW, NE = 2 * NT;
  // XCD-aware (channel, item) order: dispatch deals consecutive workgroups to the 8 XCDs in
  // turn, so the remap hands each XCD a run of consecutive channels of one item; they share
  // that item's conv-input plane x0[b] through the XCD's L2 instead of each re-fetching it
  const int Cc = C / 2, B = gridDim.y;
  int c, b;
  {
    constexpr int kXcd = 8;
    const int total = gridDim.x * gridDim.y, L = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = L % kXcd, idx = L / kXcd, q = total / kXcd, r = total % kXcd;
    const int t = xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
    b = t / gridDim.x;
    c = t - b * gridDim.x;
  }
  const float* k = coef + c * kCoef;
  const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
  const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
  const float br = k[11], bi = k[12];
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const long long HiWi = (long long)fc.Hi * fc.Wi;
  const float* x0r = fc.x0 + (long long)b * 2 * CIN * HiWi;
  const float* x0i = x0r + CIN * HiWi;
  float acc[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) acc[e] = 0.f;
  // positions i = threadIdx.x + kThreads * (U * it + u): the loads of U positions are
  // issued before any arithmetic, and (qh, qw) step incrementally (no division per position)
  constexpr int U = 4;
  int qh = threadIdx.x / W, qw = threadIdx.x - (threadIdx.x / W) * W;
  const int qstep_h = kThreads / W, qstep_w = kThreads - (kThreads / W) * W;
  auto advance = [&]() __attribute__((always_inline)) {
    qw += qstep_w;
    qh += qstep_h;
    if (qw >= W) { qw -= W; ++qh; }
  };
  auto body = [&](float fxr, float fxi, float dyr, float dyi, int ph, int pw) __attribute__((always_inline)) {
    const float xr = fxr - mr, xi = fxi - mi;
    const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
    const float g1 = dyr * act_grad(zr, act, slope) - gbr;
    const float g2 = dyi * act_grad(zi, act, slope) - gbi;
    const float gr = a00 * g1 + a01 * g2 + grr * xr + gri * xi;   // dL/dy0 (the conv's dy), never stored
    const float gi = a10 * g1 + a11 * g2 + gri * xr + gii * xi;
#pragma unroll
    for (int th = 0; th < KH; ++th) {
      const int h = ph * fc.sh + th * fc.dh - fc.ph;
      const bool hok = (unsigned)h < (unsigned)fc.Hi;
#pragma unroll
      for (int tw = 0; tw < KW; ++tw) {
        const int w = pw * fc.sw + tw * fc.dw - fc.pw;
        const bool ok = hok & ((unsigned)w < (unsigned)fc.Wi);
        const long long o = ok ? (long long)h * fc.Wi + w : 0;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const float vr = ok ? x0r[ci * HiWi + o] : 0.f;
          const float vi = ok ? x0i[ci * HiWi + o] : 0.f;
          const int e = 2 * ((ci * KH + th) * KW + tw);
          acc[e] = fmaf(gr, vr, fmaf(gi, vi, acc[e]));
          acc[e + 1] = fmaf(gi, vr, fmaf(-gr, vi, acc[e + 1]));
        }
      }
    }
  };
  int i = threadIdx.x;
  for (; i + (U - 1) * kThreads < HW; i += U * kThreads) {
    float fr[U], fm[U], dr[U], dm[U];
    int ph[U], pw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + u * kThreads;
      fr[u] = x[offr + j];
      fm[u] = x[offi + j];
      dr[u] = SRC == 1 ? gy[offr + j] + gy2[offr + j] : gy[offr + j];
      dm[u] = SRC == 1 ? gy[offi + j] + gy2[offi + j] : gy[offi + j];
      ph[u] = qh;
      pw[u] = qw;
      advance();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(fr[u], fm[u], dr[u], dm[u], ph[u], pw[u]);
  }
  for (; i < HW; i += kThreads) {
    const float dyr = SRC == 1 ? gy[offr + i] + gy2[offr + i] : gy[offr + i];
    const float dyi = SRC == 1 ? gy[offi + i] + gy2[offi + i] : gy[offi + i];
    body(x[offr + i], x[offi + i], dyr, dyi, qh, qw);
    advance();
  }
  __shared__ float red[kThreads / 64][NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const float v = se::wave_sum(acc[e]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < NE) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += red[w][threadIdx.x];
    wpart[((long long)c * B + b) * NE + threadIdx.x] = s;
  }
}

// cbn_bwd_apply_fc_kernel over CPB channels per workgroup: a position's conv-input taps
// (20 values of the spectrum at FRCRN's first conv) are loaded once and serve CPB channels,
// instead of once per channel (those L2 loads are ~80 % of the one-channel form's loads).
// grid (Cc / CPB, B); per channel the same products in the same position order as the
// one-channel form, so the partials are bit-identical.
template <int SRC, int CIN, int KH, int KW, int CPB>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply_fcm_kernel(const float* __restrict__ gy, const float* __restrict__ gy2,
                         const float* __restrict__ x, int C, int HW, int W, const float* __restrict__ coef,
                         int act, float slope, FirstConv fc, float* __restrict__ wpart) {
  static_assert(SRC == 0 || SRC == 1, "gy or gy + gy2");
  constexpr int NT = CIN * KH * KW, NE = 2 * NT;
  const int Cc = C / 2, B = gridDim.y;
  int cb, b;
  {   // XCD-aware (channel block, item) order, as cbn_bwd_apply_fc_kernel
    constexpr int kXcd = 8;
    const int total = gridDim.x * gridDim.y, L = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = L % kXcd, idx = L / kXcd, q = total / kXcd, r = total % kXcd;
    const int t = xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
    b = t / gridDim.x;
    cb = t - b * gridDim.x;
  }
  const int c0 = cb * CPB;
  const long long HiWi = (long long)fc.Hi * fc.Wi;
  const float* x0r = fc.x0 + (long long)b * 2 * CIN * HiWi;
  const float* x0i = x0r + CIN * HiWi;
  float acc[CPB][NE];
#pragma unroll
  for (int cc = 0; cc < CPB; ++cc)
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[cc][e] = 0.f;
  int qh = threadIdx.x / W, qw = threadIdx.x - (threadIdx.x / W) * W;
  const int qstep_h = kThreads / W, qstep_w = kThreads - (kThreads / W) * W;
  for (int i = threadIdx.x; i < HW; i += kThreads) {
    float vr[NT], vi[NT];
#pragma unroll
    for (int th = 0; th < KH; ++th) {
      const int h = qh * fc.sh + th * fc.dh - fc.ph;
      const bool hok = (unsigned)h < (unsigned)fc.Hi;
#pragma unroll
      for (int tw = 0; tw < KW; ++tw) {
        const int w = qw * fc.sw + tw * fc.dw - fc.pw;
        const bool ok = hok & ((unsigned)w < (unsigned)fc.Wi);
        const long long o = ok ? (long long)h * fc.Wi + w : 0;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const int tap = (ci * KH + th) * KW + tw;
          vr[tap] = ok ? x0r[ci * HiWi + o] : 0.f;
          vi[tap] = ok ? x0i[ci * HiWi + o] : 0.f;
        }
      }
    }
    float fxr[CPB], fxi[CPB], dyr[CPB], dyi[CPB];
#pragma unroll
    for (int cc = 0; cc < CPB; ++cc) {
      const long long offr = ((long long)b * C + c0 + cc) * HW, offi = ((long long)b * C + Cc + c0 + cc) * HW;
      fxr[cc] = x[offr + i];
      fxi[cc] = x[offi + i];
      dyr[cc] = SRC == 1 ? gy[offr + i] + gy2[offr + i] : gy[offr + i];
      dyi[cc] = SRC == 1 ? gy[offi + i] + gy2[offi + i] : gy[offi + i];
    }
#pragma unroll
    for (int cc = 0; cc < CPB; ++cc) {
      const float* k = coef + (c0 + cc) * kCoef;
      const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
      const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
      const float br = k[11], bi = k[12];
      const float xr = fxr[cc] - mr, xi = fxi[cc] - mi;
      const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
      const float g1 = dyr[cc] * act_grad(zr, act, slope) - gbr;
      const float g2 = dyi[cc] * act_grad(zi, act, slope) - gbi;
      const float gr = a00 * g1 + a01 * g2 + grr * xr + gri * xi;   // dL/dy0 (the conv's dy), never stored
      const float gi = a10 * g1 + a11 * g2 + gri * xr + gii * xi;
#pragma unroll
      for (int tap = 0; tap < NT; ++tap) {
        acc[cc][2 * tap] = fmaf(gr, vr[tap], fmaf(gi, vi[tap], acc[cc][2 * tap]));
        acc[cc][2 * tap + 1] = fmaf(gi, vr[tap], fmaf(-gr, vi[tap], acc[cc][2 * tap + 1]));
      }
    }
    qw += qstep_w;
    qh += qstep_h;
    if (qw >= W) { qw -= W; ++qh; }
  }
  __shared__ float red[kThreads / 64][NE];
#pragma unroll
  for (int cc = 0; cc < CPB; ++cc) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const float v = se::wave_sum(acc[cc][e]);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][e] = v;
    }
    __syncthreads();
    if (threadIdx.x < NE) {
      float sm = 0.f;
#pragma unroll
      for (int w = 0; w < kThreads / 64; ++w) sm += red[w][threadIdx.x];
      wpart[((long long)(c0 + cc) * B + b) * NE + threadIdx.x] = sm;
    }
    __syncthreads();
  }
}

// dWr / dWi[c, ci, t] = sum over the B items (fixed order, fp64) of the partials.
// grid (Cc), block NE threads
__global__ void cbn_first_conv_finish_kernel(const float* __restrict__ wpart, int B, int NE, float* dwr, float* dwi) {
  const int c = blockIdx.x, e = threadIdx.x;
  if (e >= NE) return;
  double s = 0.0;
  for (int b = 0; b < B; ++b) s += wpart[((long long)c * B + b) * NE + e];
  const int NT = NE / 2;
  (e & 1 ? dwi : dwr)[(long long)c * NT + (e >> 1)] = (float)s;
}

// Forward of the head: out[b, o, h, t] = sum_c sum_k w[o, c, k] y_c(h, t + k),
// y = act(Z (x - M) + B), t < W - 1. One thread per input position loops over
// the channels (fp32 sums in channel order, as a direct conv); a wave covers 64
// consecutive positions of one plane and writes the 63 outputs whose t + 1
// neighbour is in the wave (waves overlap by one position), taking the k = 1
// partial sum from lane + 1. grid: ceil(B * ceil(HW / 63) / 4) blocks of 256.
__global__ void __launch_bounds__(kThreads)
cbn_head_apply_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int C, int HW, int W,
                      const float* __restrict__ save, const float* __restrict__ wh, int act, float slope,
                      int64_t* nbt) {
  extern __shared__ float sm[];   // Cc x 8 CBN coefficients, then NO x C x KW head weights
  const int Cc = C / 2;
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;   // num_batches_tracked
  for (int j = threadIdx.x; j < Cc * 8; j += kThreads) {
    const int c = j >> 3, f = j & 7;
    const int src[8] = {S_MR, S_MI, S_ZRR, S_ZRI, S_ZIR, S_ZII, S_BR, S_BI};
    sm[j] = save[c * kSave + src[f]];
  }
  float* sw = sm + Cc * 8;
  for (int j = threadIdx.x; j < kHeadNO * C * kHeadKW; j += kThreads) sw[j] = wh[j];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  const int wpb = (HW + 62) / 63;   // waves per plane
  if (wave >= (long long)B * wpb) return;
  const int b = (int)(wave / wpb);
  const int pos = (int)(wave - (long long)b * wpb) * 63 + lane;
  const bool in = pos < HW;
  const float* xb = x + (long long)b * C * HW + (in ? pos : 0);
  float p[kHeadNO][kHeadKW] = {};
  constexpr int U = 4;
  for (int c0 = 0; c0 < Cc; c0 += U) {
    float vr[U], vi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(c0 + u, Cc - 1);
      vr[u] = xb[(long long)c * HW];
      vi[u] = xb[(long long)(Cc + c) * HW];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u;
      if (c < Cc) {
        const float* k = sm + c * 8;
        const float xr = vr[u] - k[0], xi = vi[u] - k[1];
        const float yr = act_fwd(k[2] * xr + k[3] * xi + k[6], act, slope);
        const float yi = act_fwd(k[4] * xr + k[5] * xi + k[7], act, slope);
#pragma unroll
        for (int o = 0; o < kHeadNO; ++o)
#pragma unroll
          for (int t = 0; t < kHeadKW; ++t)
            p[o][t] += sw[(o * C + c) * kHeadKW + t] * yr + sw[(o * C + Cc + c) * kHeadKW + t] * yi;
      }
    }
  }
  const int H = HW / W, row = pos / W, t = pos - row * W;
#pragma unroll
  for (int o = 0; o < kHeadNO; ++o) {
    const float nx = __shfl_down(p[o][1], 1, 64);   // lane + 1's k = 1 partial
    if (in && lane < 63 && t < W - 1)
      out[(((long long)b * kHeadNO + o) * H + row) * (W - 1) + t] = p[o][0] + nx;
  }
}

// moments workgroups per pass: Cc x P ~ 2048 (1024 / 4096 measured slower)
int pick_P(int B, int Cc, int HW) {
  constexpr int wg = 2048;
  const int rows = B * ((HW + kSeg - 1) / kSeg);
  return std::max(1, std::min(rows, std::max(1, wg / std::max(Cc, 1))));
}

}  // namespace

// workspace: part [Cc][P][ns] doubles, coef [Cc][kCoef], ext [Cc][P][4] floats, then
// pw_part [Cc] doubles; ns = 7 (5 forward moments, 6 backward (+1 PReLU)), or 6 +
// kHeadNS for the head's backward
static size_t ws_bytes_ns(int B, int C, int HW, int ns) {
  if (B <= 0 || C <= 0 || HW <= 0) return 0;
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  return (size_t)Cc * P * ns * sizeof(double) + (size_t)Cc * kCoef * sizeof(float) +
         (size_t)Cc * P * 4 * sizeof(float) + (size_t)Cc * sizeof(double) + 512;
}

extern "C" size_t se_cbn_workspace_size(int B, int C, int HW) { return ws_bytes_ns(B, C, HW, 7); }

extern "C" size_t se_cbn_head_workspace_size(int B, int C, int HW) {
  return ws_bytes_ns(B, C, HW, 6 + kHeadNS);
}

// the backward's workspace, then the first conv's [Cc][B][2 cin kh kw] partials
extern "C" size_t se_cbn_first_conv_workspace_size(int B, int C, int HW, int cin, int kh, int kw) {
  if (B <= 0 || C <= 0 || HW <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return 0;
  return ws_bytes_ns(B, C, HW, 7) + 256 + (size_t)(C / 2) * B * 2 * cin * kh * kw * sizeof(float);
}

// per-(channel, partition) extrema of the moments passes, after part and coef
static float* coef_of(void* ws, int Cc, int P, int ns) {
  return (float*)((char*)ws + (size_t)Cc * P * ns * sizeof(double));
}
static float* ext_of(void* ws, int Cc, int P, int ns) {
  return (float*)((char*)coef_of(ws, Cc, P, ns) + (size_t)Cc * kCoef * sizeof(float));
}
static double* pwpart_of(void* ws, int Cc, int P, int ns) {
  return (double*)(((uintptr_t)(ext_of(ws, Cc, P, ns) + (size_t)Cc * P * 4) + 7) & ~(uintptr_t)7);
}

namespace {

// moments + finalize of the training forward (running update, save, y bound)
template <typename T>
int cbn_stats(const T* x, int B, int C, int HW, const void* const* params, void* const* running,
              int64_t* nbt, float* save, int training, float eps, float momentum, float* y_amax,
              void* ws, hipStream_t st) {
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  double* part = (double*)ws;
  float* ext = ext_of(ws, Cc, P, 7);
  Ptr5 pp{};
  MPtr5 rp{};
  if (params) for (int k = 0; k < 5; ++k) pp.p[k] = params[k];
  if (running) for (int k = 0; k < 5; ++k) rp.p[k] = running[k];
  if (training) {
    hipLaunchKernelGGL(cbn_moments_kernel<T>, dim3(Cc, P), dim3(kThreads), 0, st, x, B, C, HW, P, part, ext,
                       y_amax);
    SE_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(cbn_finalize_kernel<T>, dim3(se::ceil_div(Cc, kFinWaves)), dim3(64 * kFinWaves), 0, st, part,
                     ext, P, (double)B * HW, Cc, pp, params ? 1 : 0, rp, running ? 1 : 0, (const int64_t*)nbt, save,
                     training, eps, momentum, training ? y_amax : nullptr);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

template <typename T>
int cbn_fwd_t(const T* x, T* y, int B, int C, int HW, const void* const* params, void* const* running,
              int64_t* nbt, float* save, int training, float eps, float momentum, int act, float slope,
              float* y_amax, const T* pw, void* ws, hipStream_t st) {
  const int rc = cbn_stats<T>(x, B, C, HW, params, running, nbt, save, training, eps, momentum, y_amax, ws, st);
  if (rc != SE_OK) return rc;
  int64_t* nb = (training && running) ? nbt : nullptr;
  const dim3 grid(se::ceil_div(HW, kThreads * 4), C / 2, B);
  if (HW % 4 == 0)
    hipLaunchKernelGGL(cbn_apply4_kernel<T>, grid, dim3(kThreads), 0, st, x, y, C, HW, save, act, slope, nb, pw);
  else
    hipLaunchKernelGGL(cbn_apply_kernel<T>, grid, dim3(kThreads), 0, st, x, y, C, HW, save, act, slope, nb, pw);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

bool act_ok(int act, const void* prelu_w) { return act >= 0 && act <= 2 && (!prelu_w || act == 1); }

}  // namespace

extern "C" int se_cbn_fwd(const void* x, void* y, int B, int C, int HW,
                          const void* const* params, void* const* running, int64_t* nbt,
                          float* save, int training, float eps, float momentum, int act,
                          float slope, float* y_amax, const void* prelu_w, int dtype, void* ws,
                          size_t ws_bytes, void* stream) {
  if (!x || !y || !save || B <= 0 || C <= 0 || (C & 1) || HW <= 0 || !act_ok(act, prelu_w)) return SE_E_ARG;
  if (!training && !running) return SE_E_ARG;  // eval needs running statistics
  if (ws_bytes < se_cbn_workspace_size(B, C, HW) || !ws) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  switch (dtype) {
    case SE_DTYPE_F32:
      return cbn_fwd_t<float>((const float*)x, (float*)y, B, C, HW, params, running, nbt, save, training, eps,
                              momentum, act, slope, y_amax, (const float*)prelu_w, ws, st);
    case SE_DTYPE_BF16:
      return cbn_fwd_t<__bf16>((const __bf16*)x, (__bf16*)y, B, C, HW, params, running, nbt, save, training, eps,
                               momentum, act, slope, y_amax, (const __bf16*)prelu_w, ws, st);
    case SE_DTYPE_F16:
      return cbn_fwd_t<_Float16>((const _Float16*)x, (_Float16*)y, B, C, HW, params, running, nbt, save, training,
                                 eps, momentum, act, slope, y_amax, (const _Float16*)prelu_w, ws, st);
    default:
      return SE_E_ARG;
  }
}

extern "C" int se_cbn_head_fwd(const float* x, float* out, int B, int C, int H, int W,
                               const float* const* params, float* const* running, int64_t* nbt,
                               float* save, int training, float eps, float momentum, int act,
                               float slope, const float* w_head, int out_channels, int kernel_w,
                               void* ws, size_t ws_bytes, void* stream) {
  if (!x || !out || !save || !w_head || B <= 0 || C <= 0 || (C & 1) || H <= 0 || W < 2 || act < 0 || act > 2)
    return SE_E_ARG;
  if (out_channels != kHeadNO || kernel_w != kHeadKW) return SE_E_UNSUPPORTED;
  if ((long long)H * W >= (1LL << 31)) return SE_E_UNSUPPORTED;
  if (!training && !running) return SE_E_ARG;
  const int HW = H * W;
  if (ws_bytes < se_cbn_head_workspace_size(B, C, HW) || !ws) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  const int rc = cbn_stats<float>(x, B, C, HW, (const void* const*)params, (void* const*)running, nbt, save,
                                  training, eps, momentum, nullptr, ws, st);
  if (rc != SE_OK) return rc;
  const long long waves = (long long)B * ((HW + 62) / 63);
  const size_t lds = ((size_t)(C / 2) * 8 + (size_t)kHeadNO * C * kHeadKW) * sizeof(float);
  if (lds > 64 * 1024) return SE_E_UNSUPPORTED;
  hipLaunchKernelGGL(cbn_head_apply_kernel, dim3(se::ceil_div(waves, kThreads / 64)), dim3(kThreads), lds, st,
                     x, out, B, C, HW, W, save, w_head, act, slope, (training && running) ? nbt : nullptr);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

namespace {

// src 0: gy, 1: gy + gy2, 2: the head gradient (hd). fc != NULL: the first block's
// conv weight gradient replaces the dx write (cbn_bwd_apply_fc_kernel; dx unused).
// pw / dpw: nn.PReLU's weight and its gradient (act 1 with the slope read from pw).
template <typename T>
int cbn_bwd_impl(int src, const T* gy, const T* gy2, const HeadArgs& hd, const T* x, T* dx,
                 int B, int C, int HW, const void* const* params, const float* save, void* const* dparams,
                 int training, int act, float slope, float* dx_amax, float* dwh, void* ws, size_t ws_bytes,
                 void* stream, const FirstConv* fc = nullptr, int fc_w = 0, const T* pw = nullptr,
                 T* dpw = nullptr, const CcbamDx& cd = CcbamDx{}) {
  const int ns = src == 2 ? 6 + kHeadNS : 7;   // (src 3: the 6 + 1 layout of src 0 / 1)
  if (ws_bytes < ws_bytes_ns(B, C, HW, ns) || !ws) return SE_E_WORKSPACE;
  if (pw && (src == 2 || fc || !dpw)) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  double* part = (double*)ws;
  float* coef = coef_of(ws, Cc, P, ns);
  float* ext = ext_of(ws, Cc, P, ns);
  double* pwp = pwpart_of(ws, Cc, P, ns);
  Ptr5 pp{};
  MPtr5 dp{};
  if (params) for (int k = 0; k < 5; ++k) pp.p[k] = params[k];
  if (dparams) for (int k = 0; k < 5; ++k) dp.p[k] = dparams[k];
  float* xa = training ? dx_amax : nullptr;
  const dim3 mg(Cc, P), mb(kThreads);
  const bool pr = pw != nullptr;
  if constexpr (sizeof(T) == 4) {
    if (src == 2)
      hipLaunchKernelGGL((cbn_bwd_moments_kernel<2, float>), mg, mb, 0, st, (const float*)gy, (const float*)gy2,
                         (const float*)x, B, C, HW, P, save, act, slope, part, ext, xa, hd, (const float*)nullptr,
                         CcbamDx{}, nullptr);
  }
  if constexpr (sizeof(T) == 4) {
    if (src == 3)
      hipLaunchKernelGGL((cbn_bwd_moments_kernel<3, float>), mg, mb, 0, st, (const float*)gy, (const float*)nullptr,
                         (const float*)x, B, C, HW, P, save, act, slope, part, ext, xa, hd, (const float*)nullptr, cd,
                         nullptr);
  }
  unsigned* pw_cnt = reinterpret_cast<unsigned*>(pwp + Cc);   // (within the workspace's slack)
  if (src == 1 && pr)
    hipLaunchKernelGGL((cbn_bwd_moments_kernel<1, T, true>), mg, mb, 0, st, gy, gy2, x, B, C, HW, P, save, act,
                       slope, part, ext, xa, hd, pw, CcbamDx{}, pw_cnt);
  else if (src == 1)
    hipLaunchKernelGGL((cbn_bwd_moments_kernel<1, T>), mg, mb, 0, st, gy, gy2, x, B, C, HW, P, save, act, slope,
                       part, ext, xa, hd, pw, CcbamDx{}, nullptr);
  else if (src == 0 && pr)
    hipLaunchKernelGGL((cbn_bwd_moments_kernel<0, T, true>), mg, mb, 0, st, gy, gy2, x, B, C, HW, P, save, act,
                       slope, part, ext, xa, hd, pw, CcbamDx{}, pw_cnt);
  else if (src == 0)
    hipLaunchKernelGGL((cbn_bwd_moments_kernel<0, T>), mg, mb, 0, st, gy, gy2, x, B, C, HW, P, save, act, slope,
                       part, ext, xa, hd, pw, CcbamDx{}, nullptr);
  SE_LAUNCH_CHECK();
  const dim3 fg(se::ceil_div(Cc, kFinWaves)), fb(64 * kFinWaves);
  if (src == 3 && (pr || fc || !SE_CBN_APPLY_FIN)) return SE_E_UNSUPPORTED;
  if (SE_CBN_APPLY_FIN && (src == 0 || src == 1 || src == 3) && !fc && (SE_CBN_APPLY_FIN_PR || !pr)) {
    const bool v4 = HW % 4 == 0;
    // few channels (CCBAM's one-channel spatial branch: Cc x B = 64 workgroups): each plane
    // split into segments of whole 2048-element strides, up to ~1024 workgroups
    constexpr int kStride = kThreads * 8;
    const int nseg = std::max(1, std::min(se::ceil_div(HW, kStride), 1024 / std::max(1, Cc * B)));
    const int seg_len = se::ceil_div(se::ceil_div(HW, nseg), kStride) * kStride;
    const int ns = se::ceil_div(HW, seg_len);
#define SE_AF(S, V, PRV)                                                                                              \
  hipLaunchKernelGGL((cbn_bwd_apply_fin_kernel<S, T, V, PRV>), dim3(Cc, B, ns), mb, 0, st, gy, gy2, x, dx, C, HW,      \
                     seg_len, act, slope, part, ext, P, (double)B * HW, save, pp, params ? 1 : 0, dp, dparams ? 1 : 0, \
                     training, xa, cd, pw, dpw, pwp, pw_cnt)
    if constexpr (sizeof(T) == 4) {
      if (src == 3 && v4) SE_AF(3, true, false);
      else if (src == 3) SE_AF(3, false, false);
    }
    if (src == 3) {
    } else if (pr) {
      if (src == 1 && v4) SE_AF(1, true, true);
      else if (src == 1) SE_AF(1, false, true);
      else if (v4) SE_AF(0, true, true);
      else SE_AF(0, false, true);
    } else if (src == 1 && v4) SE_AF(1, true, false);
    else if (src == 1) SE_AF(1, false, false);
    else if (v4) SE_AF(0, true, false);
    else SE_AF(0, false, false);
#undef SE_AF
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  if (src == 2)
    hipLaunchKernelGGL((cbn_bwd_finalize_kernel<true, T>), fg, fb, 0, st, part, ext, P, (double)B * HW, Cc, save, pp,
                       params ? 1 : 0, dp, dparams ? 1 : 0, training, coef, xa, dwh, pwp);
  else if (pr)
    hipLaunchKernelGGL((cbn_bwd_finalize_kernel<false, T, true>), fg, fb, 0, st, part, ext, P, (double)B * HW, Cc,
                       save, pp, params ? 1 : 0, dp, dparams ? 1 : 0, training, coef, xa, nullptr, pwp);
  else
    hipLaunchKernelGGL((cbn_bwd_finalize_kernel<false, T>), fg, fb, 0, st, part, ext, P, (double)B * HW, Cc, save,
                       pp, params ? 1 : 0, dp, dparams ? 1 : 0, training, coef, xa, nullptr, pwp);
  SE_LAUNCH_CHECK();
  if (pr) {
    hipLaunchKernelGGL(prelu_grad_finish_kernel<T>, dim3(1), dim3(64), 0, st, pwp, Cc, dpw);
    SE_LAUNCH_CHECK();
  }
  if (fc) {   // (checked by the entry point: FRCRN's first conv, cin 1, kernel (5, 2); fp32)
    if constexpr (sizeof(T) == 4) {
      float* wpart = (float*)(((uintptr_t)ws + ws_bytes_ns(B, C, HW, 7) + 255) & ~(uintptr_t)255);
      // 4 channels per workgroup where Cc % 4 == 0 (the tap-sharing form, bit-identical to the
      // one-channel cbn_bwd_apply_fc_kernel; FRCRN step 635.5 / 635.0 vs 634.0 / 631.6 utt/s)
      const int cpb = Cc % 4 == 0 ? 4 : 1;
      const float* g1 = (const float*)gy;
      const float* g2 = (const float*)gy2;
      const float* xx = (const float*)x;
#define SE_FCM(SRCV, CPBV)                                                                          \
  hipLaunchKernelGGL((cbn_bwd_apply_fcm_kernel<SRCV, 1, 5, 2, CPBV>), dim3(Cc / CPBV, B), dim3(kThreads), 0, st, \
                     g1, g2, xx, C, HW, fc_w, coef, act, slope, *fc, wpart)
      if (cpb > 1 && Cc % cpb == 0) {
        if (src == 1) SE_FCM(1, 4);
        else SE_FCM(0, 4);
      } else if (src == 1)
        hipLaunchKernelGGL((cbn_bwd_apply_fc_kernel<1, 1, 5, 2>), dim3(Cc, B), mb, 0, st, g1, g2, xx, C, HW, fc_w,
                           coef, act, slope, *fc, wpart);
      else
        hipLaunchKernelGGL((cbn_bwd_apply_fc_kernel<0, 1, 5, 2>), dim3(Cc, B), mb, 0, st, g1, g2, xx, C, HW, fc_w,
                           coef, act, slope, *fc, wpart);
#undef SE_FCM
      SE_LAUNCH_CHECK();
      hipLaunchKernelGGL(cbn_first_conv_finish_kernel, dim3(Cc), dim3(64), 0, st, wpart, B, 20, fc->dwr, fc->dwi);
      SE_LAUNCH_CHECK();
      return SE_OK;
    }
    return SE_E_UNSUPPORTED;
  }
  const dim3 grid(se::ceil_div(HW, kThreads * 4), Cc, B);
  const bool v4 = HW % 4 == 0;
  if (src == 1 && v4)
    hipLaunchKernelGGL((cbn_bwd_apply4_kernel<1, T>), grid, mb, 0, st, gy, gy2, x, dx, C, HW, coef, act, slope, pw);
  else if (src == 0 && v4)
    hipLaunchKernelGGL((cbn_bwd_apply4_kernel<0, T>), grid, mb, 0, st, gy, gy2, x, dx, C, HW, coef, act, slope, pw);
  else if (src == 1)
    hipLaunchKernelGGL((cbn_bwd_apply_kernel<1, T>), grid, mb, 0, st, gy, gy2, x, dx, C, HW, coef, act, slope, hd,
                       pw);
  else if (src == 2) {
    if constexpr (sizeof(T) == 4)
      hipLaunchKernelGGL((cbn_bwd_apply_kernel<2, float>), grid, mb, 0, st, (const float*)gy, (const float*)gy2,
                         (const float*)x, (float*)dx, C, HW, coef, act, slope, hd, (const float*)nullptr);
  } else
    hipLaunchKernelGGL((cbn_bwd_apply_kernel<0, T>), grid, mb, 0, st, gy, gy2, x, dx, C, HW, coef, act, slope, hd,
                       pw);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

bool bwd_args_ok(const void* x, const void* dx, const float* save, int B, int C, int HW) {
  return x && dx && save && B > 0 && C > 0 && !(C & 1) && HW > 0;
}

int cbn_bwd_dtype(int src, const void* gy, const void* gy2, const void* x, void* dx, int B, int C, int HW,
                  const void* const* params, const float* save, void* const* dparams, int training, int act,
                  float slope, float* dx_amax, const void* pw, void* dpw, int dtype, void* ws, size_t ws_bytes,
                  void* stream) {
  switch (dtype) {
    case SE_DTYPE_F32:
      return cbn_bwd_impl<float>(src, (const float*)gy, (const float*)gy2, HeadArgs{}, (const float*)x, (float*)dx,
                                 B, C, HW, params, save, dparams, training, act, slope, dx_amax, nullptr, ws,
                                 ws_bytes, stream, nullptr, 0, (const float*)pw, (float*)dpw);
    case SE_DTYPE_BF16:
      return cbn_bwd_impl<__bf16>(src, (const __bf16*)gy, (const __bf16*)gy2, HeadArgs{}, (const __bf16*)x,
                                  (__bf16*)dx, B, C, HW, params, save, dparams, training, act, slope, dx_amax,
                                  nullptr, ws, ws_bytes, stream, nullptr, 0, (const __bf16*)pw, (__bf16*)dpw);
    case SE_DTYPE_F16:
      return cbn_bwd_impl<_Float16>(src, (const _Float16*)gy, (const _Float16*)gy2, HeadArgs{}, (const _Float16*)x,
                                    (_Float16*)dx, B, C, HW, params, save, dparams, training, act, slope, dx_amax,
                                    nullptr, ws, ws_bytes, stream, nullptr, 0, (const _Float16*)pw, (_Float16*)dpw);
    default:
      return SE_E_ARG;
  }
}

}  // namespace

extern "C" int se_cbn_bwd(const void* gy, const void* y, const void* x, void* dx, int B,
                          int C, int HW, const void* const* params, const float* save,
                          void* const* dparams, int training, int act, float slope,
                          float* dx_amax, const void* prelu_w, void* dprelu_w, int dtype, void* ws, size_t ws_bytes,
                          void* stream) {
  (void)y;   // not read: act' is recomputed from x (see the file comment); may be NULL
  if (!gy || !bwd_args_ok(x, dx, save, B, C, HW) || !act_ok(act, prelu_w)) return SE_E_ARG;
  return cbn_bwd_dtype(0, gy, nullptr, x, dx, B, C, HW, params, save, dparams, training, act, slope, dx_amax,
                       prelu_w, dprelu_w, dtype, ws, ws_bytes, stream);
}

// Forked output (the encoder block's y feeds the next conv AND the decoder skip):
// gy + gy2 is summed inside both passes instead of by a separate add of two
// activation-sized tensors (3 passes) before the backward.
extern "C" int se_cbn_bwd2(const void* gy, const void* gy2, const void* x, void* dx, int B,
                           int C, int HW, const void* const* params, const float* save,
                           void* const* dparams, int training, int act, float slope,
                           float* dx_amax, const void* prelu_w, void* dprelu_w, int dtype, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!gy || !gy2 || !bwd_args_ok(x, dx, save, B, C, HW) || !act_ok(act, prelu_w)) return SE_E_ARG;
  return cbn_bwd_dtype(1, gy, gy2, x, dx, B, C, HW, params, save, dparams, training, act, slope, dx_amax,
                       prelu_w, dprelu_w, dtype, ws, ws_bytes, stream);
}

// Forked output whose second consumer is FRCRN's CCBAM skip gate: gy + the gate's input
// gradient formed inside both passes from its parts (CcbamDx), so the gate's dx tensor is
// never written (ccbam.hip bwd_dx_kernel: one read and one write of the skip per layer).
extern "C" int se_cbn_bwd_ccbam(const float* gy, const float* g_gate, const float* dP, const short* idx,
                                const float* ca, const float* dmean, const float* dmax, const int* amax,
                                const float* x, float* dx, int B, int C, int HW, const float* const* params,
                                const float* save, float* const* dparams, int training, int act, float slope,
                                float* dx_amax, void* ws, size_t ws_bytes, void* stream) {
  if (!gy || !g_gate || !dP || !idx || !ca || !dmean || !dmax || !amax) return SE_E_ARG;
  if (!bwd_args_ok(x, dx, save, B, C, HW) || act < 0 || act > 2) return SE_E_ARG;
  if (C / 2 > 32767) return SE_E_SHAPE;
  const CcbamDx cd{g_gate, dP, idx, ca, dmean, dmax, amax};
  return cbn_bwd_impl<float>(3, gy, nullptr, HeadArgs{}, x, dx, B, C, HW, (const void* const*)params, save,
                             (void* const*)dparams, training, act, slope, dx_amax, nullptr, ws, ws_bytes, stream,
                             nullptr, 0, nullptr, nullptr, cd);
}

extern "C" int se_cbn_head_bwd(const float* gout, const float* x, float* dx, int B, int C, int H, int W,
                               const float* const* params, const float* save, float* const* dparams,
                               const float* w_head, float* dw_head, int out_channels, int kernel_w,
                               int training, int act, float slope, float* dx_amax, void* ws,
                               size_t ws_bytes, void* stream) {
  if (!gout || !w_head || !dw_head || H <= 0 || W < 2 || act < 0 || act > 2) return SE_E_ARG;
  if (out_channels != kHeadNO || kernel_w != kHeadKW) return SE_E_UNSUPPORTED;
  if ((long long)H * W >= (1LL << 31)) return SE_E_UNSUPPORTED;
  if (!bwd_args_ok(x, dx, save, B, C, H * W)) return SE_E_ARG;
  const HeadArgs hd{gout, w_head, W};
  return cbn_bwd_impl<float>(2, nullptr, nullptr, hd, x, dx, B, C, H * W, (const void* const*)params, save,
                             (void* const*)dparams, training, act, slope, dx_amax, dw_head, ws, ws_bytes, stream);
}

// First block (conv -> ComplexBatchNorm2d + act) with a conv input that needs no
// gradient: the CBN backward with the conv's weight gradient accumulated in the
// apply pass instead of writing dL/dy0 (see cbn_bwd_apply_fc_kernel).
extern "C" int se_cbn_bwd_first_conv(const float* gy, const float* gy2, const float* x, int B, int C, int H, int W,
                                     const float* const* params, const float* save, float* const* dparams,
                                     int training, int act, float slope, const se_first_conv* fc, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (!gy || !fc || !fc->x0 || !fc->dwr || !fc->dwi || H <= 0 || W <= 0 || act < 0 || act > 2) return SE_E_ARG;
  if (!bwd_args_ok(x, x, save, B, C, H * W)) return SE_E_ARG;
  if (fc->cin != 1 || fc->kernel_h != 5 || fc->kernel_w != 2) return SE_E_UNSUPPORTED;
  if (fc->in_h <= 0 || fc->in_w <= 0 || fc->stride_h <= 0 || fc->stride_w <= 0 || fc->dil_h <= 0 || fc->dil_w <= 0)
    return SE_E_ARG;
  if ((long long)fc->in_h * fc->in_w * 2 >= (1LL << 31) || (long long)H * W >= (1LL << 31)) return SE_E_UNSUPPORTED;
  if (ws_bytes < se_cbn_first_conv_workspace_size(B, C, H * W, fc->cin, fc->kernel_h, fc->kernel_w) || !ws)
    return SE_E_WORKSPACE;
  const FirstConv f{fc->x0, fc->in_h, fc->in_w, fc->stride_h, fc->stride_w, fc->pad_h, fc->pad_w, fc->dil_h,
                    fc->dil_w, fc->dwr, fc->dwi};
  return cbn_bwd_impl<float>(gy2 ? 1 : 0, gy, gy2, HeadArgs{}, x, nullptr, B, C, H * W, (const void* const*)params,
                             save, (void* const*)dparams, training, act, slope, nullptr, nullptr, ws, ws_bytes, stream,
                             &f, W);
}
