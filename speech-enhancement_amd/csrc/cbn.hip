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

namespace {

constexpr int kThreads = 256;
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

struct Ptr5 { const float* p[5]; };
struct MPtr5 { float* p[5]; };

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

__device__ __forceinline__ float act_grad(float y, int act, float slope) {
  if (act == 1) return y > 0.f ? 1.f : slope;
  if (act == 2) return y > 0.f ? 1.f : 0.f;
  return 1.f;
}

// grid (Cc, P). Row r = (b, segment) of channel c; rows strided over P.
// ext[(c * P + p) * 4 + {0..3}] = max x_r, -min x_r, max x_i, -min x_i
__global__ void __launch_bounds__(kThreads)
cbn_moments_kernel(const float* __restrict__ x, int B, int C, int HW, int P, double* part, float* ext,
                   float* y_amax) {
  const int Cc = C / 2, c = blockIdx.x, p = blockIdx.y;
  if (y_amax && c == 0 && p == 0 && threadIdx.x == 0) *y_amax = 0.f;   // the finalize blocks atomicMax into it
  const int nseg = (HW + kSeg - 1) / kSeg;
  double v[5] = {0, 0, 0, 0, 0};
  float e[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int row = p; row < B * nseg; row += P) {
    const int b = row / nseg, sg = row - b * nseg;
    const float* xr = x + ((long long)b * C + c) * HW;
    const float* xi = x + ((long long)b * C + Cc + c) * HW;
    const int i1 = min(HW, (sg + 1) * kSeg);
    for (int i = sg * kSeg + threadIdx.x; i < i1; i += kThreads) {
      const float fr = xr[i], fm = xi[i];
      e[0] = fmaxf(e[0], fr); e[1] = fmaxf(e[1], -fr); e[2] = fmaxf(e[2], fm); e[3] = fmaxf(e[3], -fm);
      const double r = fr, m = fm;
      v[0] += r; v[1] += m; v[2] += r * r; v[3] += r * m; v[4] += m * m;
    }
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
        float* rm[5] = {running.p[0], running.p[1], running.p[2], running.p[3], running.p[4]};
        const float nv[5] = {(float)mr, (float)mi, (float)vrr, (float)vri, (float)vii};
        for (int k = 0; k < 5; ++k) rm[k][c] = rm[k][c] + factor * (nv[k] - rm[k][c]);
      }
    } else {
      mr = running.p[0][c]; mi = running.p[1][c];
      vrr = running.p[2][c]; vri = running.p[3][c]; vii = running.p[4][c];
    }
    vrr += eps; vii += eps;
    const double s = sqrt(vrr * vii - vri * vri);
    const double t = sqrt(vrr + vii + 2.0 * s);
    const double r = 1.0 / (s * t);
    const double urr = (s + vii) * r, uii = (s + vrr) * r, uri = -vri * r;
    double zrr = urr, zri = uri, zir = uri, zii = uii, br = 0, bi = 0;
    if (affine) {
      const double wrr = params.p[0][c], wri = params.p[1][c], wii = params.p[2][c];
      zrr = wrr * urr + wri * uri;
      zri = wrr * uri + wri * uii;
      zir = wri * urr + wii * uri;
      zii = wri * uri + wii * uii;
      br = params.p[3][c]; bi = params.p[4][c];
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

// grid (ceil(HW / (kThreads*4)), Cc, B)
__global__ void __launch_bounds__(kThreads)
cbn_apply_kernel(const float* __restrict__ x, float* __restrict__ y, int C, int HW,
                 const float* __restrict__ save, int act, float slope, int64_t* nbt) {
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  if (nbt && blockIdx.x == 0 && c == 0 && b == 0 && threadIdx.x == 0) *nbt += 1;   // num_batches_tracked
  const float* s = save + c * kSave;
  const float mr = s[S_MR], mi = s[S_MI], zrr = s[S_ZRR], zri = s[S_ZRI];
  const float zir = s[S_ZIR], zii = s[S_ZII], br = s[S_BR], bi = s[S_BI];
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int base = blockIdx.x * kThreads * 4 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = base + u * kThreads;
    if (i < HW) {
      const float xr = x[offr + i] - mr, xi = x[offi + i] - mi;
      float yr = zrr * xr + zri * xi + br;
      float yi = zir * xr + zii * xi + bi;
      if (act == 1) { yr = yr > 0.f ? yr : yr * slope; yi = yi > 0.f ? yi : yi * slope; }
      else if (act == 2) { yr = fmaxf(yr, 0.f); yi = fmaxf(yi, 0.f); }
      y[offr + i] = yr;
      y[offi + i] = yi;
    }
  }
}

// Backward moments: g = (gy [+ gy2]) * act'(z), xt = x - M. gy2 (G2) is a second
// gradient of the same output (a forked output, se_cbn_bwd2): summed on the fly.
// sums: gr, gi, gr*xtr, gr*xti, gi*xtr, gi*xti
template <bool G2>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_moments_kernel(const float* __restrict__ gy, const float* __restrict__ gy2,
                       const float* __restrict__ x, int B, int C, int HW, int P,
                       const float* __restrict__ save, int act, float slope, double* part, float* ext,
                       float* dx_amax) {
  const int Cc = C / 2, c = blockIdx.x, p = blockIdx.y;
  if (dx_amax && c == 0 && p == 0 && threadIdx.x == 0) *dx_amax = 0.f;   // the finalize blocks atomicMax into it
  const int nseg = (HW + kSeg - 1) / kSeg;
  const float* sv = save + c * kSave;
  float gmr = 0.f, gmi = 0.f;   // max |g_r|, max |g_i| (the dx bound)
  const float mr = sv[S_MR], mi = sv[S_MI];
  const float zrr = sv[S_ZRR], zri = sv[S_ZRI], zir = sv[S_ZIR], zii = sv[S_ZII], br = sv[S_BR], bi = sv[S_BI];
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (int row = p; row < B * nseg; row += P) {
    const int b = row / nseg, sg = row - b * nseg;
    const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
    const int i1 = min(HW, (sg + 1) * kSeg);
    for (int i = sg * kSeg + threadIdx.x; i < i1; i += kThreads) {
      const float xr = x[offr + i] - mr, xi = x[offi + i] - mi;
      const float zr = zrr * xr + zri * xi + br, zi = zir * xr + zii * xi + bi;   // = forward pre-activation
      const float gr = (G2 ? gy[offr + i] + gy2[offr + i] : gy[offr + i]) * act_grad(zr, act, slope);
      const float gi = (G2 ? gy[offi + i] + gy2[offi + i] : gy[offi + i]) * act_grad(zi, act, slope);
      gmr = fmaxf(gmr, fabsf(gr)); gmi = fmaxf(gmi, fabsf(gi));
      v[0] += gr; v[1] += gi;
      v[2] += (double)gr * xr; v[3] += (double)gr * xi;
      v[4] += (double)gi * xr; v[5] += (double)gi * xi;
    }
  }
  block_reduce_store<6>(v, part + ((long long)c * P + p) * 6);
  __syncthreads();
  gmr = block_max(gmr);
  __syncthreads();
  gmi = block_max(gmi);
  if (threadIdx.x == 0) {
    ext[((long long)c * P + p) * 2 + 0] = gmr;
    ext[((long long)c * P + p) * 2 + 1] = gmi;
  }
}

// coef layout per channel (16 floats): ZTrr ZTri ZTir ZTii gbr gbi Grr Gri Gii Mr Mi Br Bi pad
constexpr int kCoef = 16;

// One wave per channel, as cbn_finalize_kernel; the bound of max |dx| goes to
// *dx_amax by atomicMax (zeroed by the backward moments pass).
__global__ void __launch_bounds__(64 * kFinWaves)
cbn_bwd_finalize_kernel(const double* part, const float* ext, int P, double count, int Cc,
                        const float* save, Ptr5 params, int affine,
                        MPtr5 dparams, int has_dparams, int training,
                        float* coef, float* dx_amax) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (c >= Cc) return;
  double sm[6] = {0, 0, 0, 0, 0, 0};
  float gmr = 0.f, gmi = 0.f;
  for (int p = lane; p < P; p += 64) {
#pragma unroll
    for (int k = 0; k < 6; ++k) sm[k] += part[((long long)c * P + p) * 6 + k];
    gmr = fmaxf(gmr, ext[((long long)c * P + p) * 2 + 0]);
    gmi = fmaxf(gmi, ext[((long long)c * P + p) * 2 + 1]);
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) sm[k] = se::wave_sum(sm[k]);
  gmr = se::wave_max(gmr);
  gmi = se::wave_max(gmi);
  if (lane != 0) return;
  {
    const float* s = save + (long long)c * kSave;
    const double urr = s[S_URR], uri = s[S_URI], uii = s[S_UII];
    const double vrr = s[S_VRR], vri = s[S_VRI], vii = s[S_VII];
    const double ss = s[S_S], tt = s[S_T];
    // dZ = sum g xt^T
    const double dz00 = sm[2], dz01 = sm[3], dz10 = sm[4], dz11 = sm[5];
    double wrr = 1, wri = 0, wii = 1;
    if (affine) { wrr = params.p[0][c]; wri = params.p[1][c]; wii = params.p[2][c]; }
    double gurr, guri, guii;
    if (affine) {
      // dW = dZ U (U symmetric); W symmetric -> Wri collects both off-diagonals
      const double dw00 = dz00 * urr + dz01 * uri, dw01 = dz00 * uri + dz01 * uii;
      const double dw10 = dz10 * urr + dz11 * uri, dw11 = dz10 * uri + dz11 * uii;
      if (has_dparams) {
        dparams.p[0][c] = (float)dw00;
        dparams.p[1][c] = (float)(dw01 + dw10);
        dparams.p[2][c] = (float)dw11;
        dparams.p[3][c] = (float)sm[0];
        dparams.p[4][c] = (float)sm[1];
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
    float* o = coef + (long long)c * kCoef;
    o[0] = (float)zrr; o[1] = (float)zir;   // dxr = Zrr g_r + Zir g_i
    o[2] = (float)zri; o[3] = (float)zii;   // dxi = Zri g_r + Zii g_i
    o[4] = (float)gbr; o[5] = (float)gbi;
    o[6] = (float)grr; o[7] = (float)gri; o[8] = (float)gii;
    o[9] = s[S_MR]; o[10] = s[S_MI]; o[11] = s[S_BR]; o[12] = s[S_BI];
    o[13] = o[14] = o[15] = 0.f;
    if (training && dx_amax) {   // dx = Z^T (g - gb) + Gamma (x - M), bounded term by term
      const float gr = gmr + fabsf(o[4]);
      const float gi = gmi + fabsf(o[5]);
      const float dr = s[S_DR], di = s[S_DI];
      const float br = fabsf(o[0]) * gr + fabsf(o[1]) * gi + fabsf(o[6]) * dr + fabsf(o[7]) * di;
      const float bi = fabsf(o[2]) * gr + fabsf(o[3]) * gi + fabsf(o[7]) * dr + fabsf(o[8]) * di;
      atomicMax(reinterpret_cast<unsigned*>(dx_amax), __float_as_uint(fmaxf(br, bi) * 1.0001f));
    }
  }
}

template <bool G2>
__global__ void __launch_bounds__(kThreads)
cbn_bwd_apply_kernel(const float* __restrict__ gy, const float* __restrict__ gy2,
                     const float* __restrict__ x, float* __restrict__ dx, int C, int HW,
                     const float* __restrict__ coef, int act, float slope) {
  const int Cc = C / 2, c = blockIdx.y, b = blockIdx.z;
  const float* k = coef + c * kCoef;
  const float a00 = k[0], a01 = k[1], a10 = k[2], a11 = k[3];
  const float gbr = k[4], gbi = k[5], grr = k[6], gri = k[7], gii = k[8], mr = k[9], mi = k[10];
  const float br = k[11], bi = k[12];
  // forward Z = [[a00, a10], [a01, a11]] (coef holds Z^T)
  const long long offr = ((long long)b * C + c) * HW, offi = ((long long)b * C + Cc + c) * HW;
  const int base = blockIdx.x * kThreads * 4 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = base + u * kThreads;
    if (i < HW) {
      const float xr = x[offr + i] - mr, xi = x[offi + i] - mi;
      const float zr = a00 * xr + a10 * xi + br, zi = a01 * xr + a11 * xi + bi;   // = forward pre-activation
      const float gr = (G2 ? gy[offr + i] + gy2[offr + i] : gy[offr + i]) * act_grad(zr, act, slope) - gbr;
      const float gi = (G2 ? gy[offi + i] + gy2[offi + i] : gy[offi + i]) * act_grad(zi, act, slope) - gbi;
      dx[offr + i] = a00 * gr + a01 * gi + grr * xr + gri * xi;
      dx[offi + i] = a10 * gr + a11 * gi + gri * xr + gii * xi;
    }
  }
}

int pick_P(int B, int Cc, int HW) {
  const int rows = B * ((HW + kSeg - 1) / kSeg);
  return std::max(1, std::min(rows, std::max(1, 2048 / std::max(Cc, 1))));
}

}  // namespace

extern "C" size_t se_cbn_workspace_size(int B, int C, int HW) {
  if (B <= 0 || C <= 0 || HW <= 0) return 0;
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  return (size_t)Cc * P * 6 * sizeof(double) + (size_t)Cc * kCoef * sizeof(float) +
         (size_t)Cc * P * 4 * sizeof(float) + 512;
}

// per-(channel, partition) extrema of the moments passes, after part and coef
static float* ext_of(void* ws, int Cc, int P) {
  return (float*)((char*)ws + (size_t)Cc * P * 6 * sizeof(double) + (size_t)Cc * kCoef * sizeof(float));
}

extern "C" int se_cbn_fwd(const float* x, float* y, int B, int C, int HW,
                          const float* const* params, float* const* running, int64_t* nbt,
                          float* save, int training, float eps, float momentum, int act,
                          float slope, float* y_amax, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !y || !save || B <= 0 || C <= 0 || (C & 1) || HW <= 0 || act < 0 || act > 2)
    return SE_E_ARG;
  if (!training && !running) return SE_E_ARG;  // eval needs running statistics
  if (ws_bytes < se_cbn_workspace_size(B, C, HW) || !ws) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  double* part = (double*)ws;
  float* ext = ext_of(ws, Cc, P);
  Ptr5 pp{};
  MPtr5 rp{};
  if (params) for (int k = 0; k < 5; ++k) pp.p[k] = params[k];
  if (running) for (int k = 0; k < 5; ++k) rp.p[k] = running[k];
  if (training) {
    hipLaunchKernelGGL(cbn_moments_kernel, dim3(Cc, P), dim3(kThreads), 0, st, x, B, C, HW, P, part, ext,
                       y_amax);
    SE_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(cbn_finalize_kernel, dim3(se::ceil_div(Cc, kFinWaves)), dim3(64 * kFinWaves), 0, st, part,
                     ext, P, (double)B * HW, Cc, pp, params ? 1 : 0, rp, running ? 1 : 0, (const int64_t*)nbt, save,
                     training, eps, momentum, training ? y_amax : nullptr);
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(cbn_apply_kernel, dim3(se::ceil_div(HW, kThreads * 4), Cc, B), dim3(kThreads),
                     0, st, x, y, C, HW, save, act, slope, (training && running) ? nbt : nullptr);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

namespace {

int cbn_bwd_impl(const float* gy, const float* gy2, const float* x, float* dx, int B, int C,
                 int HW, const float* const* params, const float* save, float* const* dparams,
                 int training, int act, float slope, float* dx_amax, void* ws, size_t ws_bytes,
                 void* stream) {
  if (!gy || !x || !dx || !save || B <= 0 || C <= 0 || (C & 1) || HW <= 0) return SE_E_ARG;
  if (ws_bytes < se_cbn_workspace_size(B, C, HW) || !ws) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  const int Cc = C / 2;
  const int P = pick_P(B, Cc, HW);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + (size_t)Cc * P * 6 * sizeof(double));
  float* ext = ext_of(ws, Cc, P);
  Ptr5 pp{};
  MPtr5 dp{};
  if (params) for (int k = 0; k < 5; ++k) pp.p[k] = params[k];
  if (dparams) for (int k = 0; k < 5; ++k) dp.p[k] = dparams[k];
  if (gy2)
    hipLaunchKernelGGL(cbn_bwd_moments_kernel<true>, dim3(Cc, P), dim3(kThreads), 0, st, gy, gy2, x,
                       B, C, HW, P, save, act, slope, part, ext, training ? dx_amax : nullptr);
  else
    hipLaunchKernelGGL(cbn_bwd_moments_kernel<false>, dim3(Cc, P), dim3(kThreads), 0, st, gy, gy2,
                       x, B, C, HW, P, save, act, slope, part, ext, training ? dx_amax : nullptr);
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(cbn_bwd_finalize_kernel, dim3(se::ceil_div(Cc, kFinWaves)), dim3(64 * kFinWaves), 0, st,
                     part, ext, P, (double)B * HW, Cc, save, pp, params ? 1 : 0, dp, dparams ? 1 : 0, training,
                     coef, training ? dx_amax : nullptr);
  SE_LAUNCH_CHECK();
  const dim3 grid(se::ceil_div(HW, kThreads * 4), Cc, B);
  if (gy2)
    hipLaunchKernelGGL(cbn_bwd_apply_kernel<true>, grid, dim3(kThreads), 0, st, gy, gy2, x, dx, C,
                       HW, coef, act, slope);
  else
    hipLaunchKernelGGL(cbn_bwd_apply_kernel<false>, grid, dim3(kThreads), 0, st, gy, gy2, x, dx, C,
                       HW, coef, act, slope);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

}  // namespace

extern "C" int se_cbn_bwd(const float* gy, const float* y, const float* x, float* dx, int B,
                          int C, int HW, const float* const* params, const float* save,
                          float* const* dparams, int training, int act, float slope,
                          float* dx_amax, void* ws, size_t ws_bytes, void* stream) {
  (void)y;   // not read: act' is recomputed from x (see the file comment); may be NULL
  return cbn_bwd_impl(gy, nullptr, x, dx, B, C, HW, params, save, dparams, training, act, slope,
                      dx_amax, ws, ws_bytes, stream);
}

// Forked output (the encoder block's y feeds the next conv AND the decoder skip):
// gy + gy2 is summed inside both passes instead of by a separate add of two
// activation-sized tensors (3 passes) before the backward.
extern "C" int se_cbn_bwd2(const float* gy, const float* gy2, const float* x, float* dx, int B,
                           int C, int HW, const float* const* params, const float* save,
                           float* const* dparams, int training, int act, float slope,
                           float* dx_amax, void* ws, size_t ws_bytes, void* stream) {
  if (!gy2) return SE_E_ARG;
  return cbn_bwd_impl(gy, gy2, x, dx, B, C, HW, params, save, dparams, training, act, slope,
                      dx_amax, ws, ws_bytes, stream);
}
