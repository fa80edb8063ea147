// Fused complex CBAM skip attention (reference: models/modules/ccbam.py:28-106).
//
//   ca  = sigmoid(MLP(avgpool_hw(x)) + MLP(maxpool_hw(x)))          [B, C]
//   x1  = x * ca
//   P   = [mean_c(x1_re), max_c(x1_re), mean_c(x1_im), max_c(x1_im)] [B, 4, HW]
//   sa  = sigmoid(ReLU(CBN(ComplexConv2d(4->2, k7)(P))))            [B, 2, HW]
//   out = x1 + sa[:, half(c)]
//
// The MLP and the 4->2 conv/CBN are small and stay in their own modules; the
// five kernels here are the passes over the full [B, C, HW] skip tensor, each
// one HBM-bound read/write stream:
//   fwd: channel_pool (1R), spatial_pool (1R), apply (1R 1W)
//   bwd: bwd_sa (1R), bwd_dca (2R), bwd_dx (1R 1W)
// against ~25 passes for the unfused PyTorch graph. Max-pool gradients go to
// the FIRST maximal index, like AdaptiveMaxPool2d / torch.max(dim) in the
// reference (torch.amax would split them among ties).
//
// Complex layout (complex_nn.py:18-42): channels [0, C/2) real, [C/2, C) imag.
#include "common.hpp"

namespace {

constexpr int kThreads = 256;

// ---------------------------------------------------------------- forward
// one block per (b, c): mean, max and first argmax over HW
__global__ __launch_bounds__(kThreads) void channel_pool_kernel(const float* __restrict__ x, float* __restrict__ mean,
                                                                float* __restrict__ mx, int* __restrict__ amax, int HW) {
  const size_t row = blockIdx.x;
  const float* p = x + row * HW;
  // four independent chains (more loads in flight); chain k sees ascending
  // indices, so keeping the first maximum per chain and merging by index is
  // exact first-argmax semantics
  float s4[4] = {0.f, 0.f, 0.f, 0.f}, m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int i4[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
  int i = threadIdx.x;
  for (; i + 3 * kThreads < HW; i += 4 * kThreads) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[i + k * kThreads];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s4[k] += v[k];
      if (v[k] > m4[k]) { m4[k] = v[k]; i4[k] = i + k * kThreads; }
    }
  }
  for (int k = 0; i < HW; i += kThreads, ++k) {
    const float v = p[i];
    s4[k] += v;
    if (v > m4[k]) { m4[k] = v; i4[k] = i; }
  }
  float s = (s4[0] + s4[1]) + (s4[2] + s4[3]), m = m4[0];
  int mi = i4[0];
#pragma unroll
  for (int k = 1; k < 4; ++k)
    if (m4[k] > m || (m4[k] == m && i4[k] < mi)) { m = m4[k]; mi = i4[k]; }
  // wave reduce (sum; max with smallest index on ties)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    const float m2 = __shfl_xor(m, o, 64);
    const int i2 = __shfl_xor(mi, o, 64);
    if (m2 > m || (m2 == m && i2 < mi)) { m = m2; mi = i2; }
  }
  __shared__ float ss[kThreads / 64], sm[kThreads / 64];
  __shared__ int si[kThreads / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { ss[w] = s; sm[w] = m; si[w] = mi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = ss[0], M = sm[0];
    int I = si[0];
    for (int k = 1; k < kThreads / 64; ++k) {
      S += ss[k];
      if (sm[k] > M || (sm[k] == M && si[k] < I)) { M = sm[k]; I = si[k]; }
    }
    mean[row] = S / (float)HW;
    mx[row] = M;
    amax[row] = I;
  }
}

// thread per (b, hw): channel mean / max / first argmax of x*ca within each half
__global__ __launch_bounds__(kThreads) void spatial_pool_kernel(const float* __restrict__ x, const float* __restrict__ ca,
                                                                float* __restrict__ P, short* __restrict__ idx, int C,
                                                                int HW) {
  const int b = blockIdx.y;
  const int hw = blockIdx.x * kThreads + threadIdx.x;
  extern __shared__ float sca[];
  for (int c = threadIdx.x; c < C; c += kThreads) sca[c] = ca[(size_t)b * C + c];
  __syncthreads();
  if (hw >= HW) return;
  const int Ch = C / 2;
  const float* xb = x + (size_t)b * C * HW + hw;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float s = 0.f, m = -INFINITY;
    int mi = 0;
    for (int c = 0; c < Ch; ++c) {
      const float v = xb[(size_t)(h * Ch + c) * HW] * sca[h * Ch + c];
      s += v;
      if (v > m) { m = v; mi = c; }
    }
    P[((size_t)b * 4 + 2 * h) * HW + hw] = s / (float)Ch;
    P[((size_t)b * 4 + 2 * h + 1) * HW + hw] = m;
    idx[((size_t)b * 2 + h) * HW + hw] = (short)mi;
  }
}

// out = x*ca + sa[half]; with amax (ABI 10), also max |out| (atomic max of the fp32 bit
// patterns into the slot the entry point zeroed): the SE_MATH_F16X3 scale source of the
// GEMMs that read out, exact instead of the bound max |x| + 1
__global__ __launch_bounds__(kThreads) void apply_kernel(const float* __restrict__ x, const float* __restrict__ ca,
                                                         const float* __restrict__ sa, float* __restrict__ out, int C,
                                                         int HW, unsigned* __restrict__ amax) {
  const int b = blockIdx.y;
  const int hw = blockIdx.x * kThreads + threadIdx.x;
  extern __shared__ float sca[];
  for (int c = threadIdx.x; c < C; c += kThreads) sca[c] = ca[(size_t)b * C + c];
  __syncthreads();
  float m = 0.f;
  if (hw < HW) {
    const int Ch = C / 2;
    const float s0 = sa[((size_t)b * 2) * HW + hw], s1 = sa[((size_t)b * 2 + 1) * HW + hw];
    const size_t base = (size_t)b * C * HW + hw;
#pragma unroll 8
    for (int c = 0; c < C; ++c) {
      const float v = x[base + (size_t)c * HW] * sca[c] + (c < Ch ? s0 : s1);
      out[base + (size_t)c * HW] = v;
      m = fmaxf(m, fabsf(v));
    }
  }
  if (amax) {
    const unsigned bits = __builtin_bit_cast(unsigned, se::wave_max(m));
    if ((threadIdx.x & 63) == 0 && bits) atomicMax(amax, bits);
  }
}

// ---------------------------------------------------------------- backward
// dsa[b, h, hw] = sum_{c in half h} gout[b, c, hw]
__global__ __launch_bounds__(kThreads) void bwd_sa_kernel(const float* __restrict__ g, float* __restrict__ dsa, int C,
                                                          int HW) {
  const int b = blockIdx.y;
  const int hw = blockIdx.x * kThreads + threadIdx.x;
  if (hw >= HW) return;
  const int Ch = C / 2;
  const float* gb = g + (size_t)b * C * HW + hw;
  float s0 = 0.f, s1 = 0.f;
  // eight loads per half in flight; each half still sums in channel order
  constexpr int U = 8;
  int c = 0;
  for (; c + U <= Ch; c += U) {
    float v0[U], v1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v0[u] = gb[(size_t)(c + u) * HW];
      v1[u] = gb[(size_t)(Ch + c + u) * HW];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { s0 += v0[u]; s1 += v1[u]; }
  }
  for (; c < Ch; ++c) { s0 += gb[(size_t)c * HW]; s1 += gb[(size_t)(Ch + c) * HW]; }
  dsa[((size_t)b * 2) * HW + hw] = s0;
  dsa[((size_t)b * 2 + 1) * HW + hw] = s1;
}

// Per (b, c): dca = sum_hw gx1 * x with gx1 = gout + dP_avg/Ch + [c is the
// spatial argmax] * dP_max (the full gradient reaching x1 = x*ca). Blocks are
// (tile of kPos*256 positions, group of kCG channels, b): kCG independent
// accumulators, all kCG*kPos*2 loads of a thread issued together; per-tile
// channel partials are summed by dca_reduce_kernel (fixed order).
constexpr int kPos = 4;
template <int kCG>
__global__ __launch_bounds__(kThreads) void bwd_dca_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                           const float* __restrict__ dP, const short* __restrict__ idx,
                                                           float* __restrict__ part, int C, int HW, int ntiles) {
  const int tile = blockIdx.x, c0 = blockIdx.y * kCG, b = blockIdx.z;
  const int Ch = C / 2;
  const int h = c0 < Ch ? 0 : 1;                    // kCG divides Ch: a group never straddles halves
  const float inv = 1.f / (float)Ch;
  float pa[kPos], pm[kPos], ok[kPos];
  int pi[kPos], hwc[kPos];
#pragma unroll
  for (int j = 0; j < kPos; ++j) {
    const int hw = (tile * kPos + j) * kThreads + threadIdx.x;
    ok[j] = hw < HW ? 1.f : 0.f;
    hwc[j] = hw < HW ? hw : HW - 1;                 // clamped: branch-free loads, zero weight
    pa[j] = dP[((size_t)b * 4 + 2 * h) * HW + hwc[j]] * inv;
    pm[j] = dP[((size_t)b * 4 + 2 * h + 1) * HW + hwc[j]];
    pi[j] = idx[((size_t)b * 2 + h) * HW + hwc[j]];
  }
  float acc[kCG];
  const size_t base = ((size_t)b * C + c0) * HW;
#pragma unroll
  for (int k = 0; k < kCG; ++k) {
    const int cc = c0 + k - h * Ch;
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < kPos; ++j) {
      const size_t o = base + (size_t)k * HW + hwc[j];
      const float gx = g[o] + pa[j] + (pi[j] == cc ? pm[j] : 0.f);
      a += ok[j] * (gx * x[o]);
    }
    acc[k] = a;
  }
  __shared__ float sred[kThreads / 64][kCG];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kCG; ++k) {
    const float v = se::wave_sum(acc[k]);
    if (lane == 0) sred[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < kCG) {
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < kThreads / 64; ++q) sum += sred[q][threadIdx.x];
    part[((size_t)b * ntiles + tile) * C + c0 + threadIdx.x] = sum;
  }
}

__global__ void dca_reduce_kernel(const float* __restrict__ part, float* __restrict__ dca, int B, int C, int ntiles) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i % C;
  float s = 0.f;
  for (int t = 0; t < ntiles; ++t) s += part[((size_t)b * ntiles + t) * C + c];
  dca[i] = s;
}

// The spatial gate's sigmoid backward fused into the channel sums (the gate sa =
// sigmoid(z) of the spatial branch, ccbam.py:82-86): dz[b, h, hw] =
// (sum_{c in half h} gout[b, c, hw]) * (1 - sa) * sa, the sums in channel order
// and the product in ATen's sigmoid_backward order, so dz is bit-identical to
// bwd_sa_kernel followed by torch's sigmoid backward. Four consecutive positions
// per thread (16-B loads when HW % 4 == 0): a block streams 4-KB segments of each
// channel plane instead of 1 KB.
typedef float f32x4c __attribute__((ext_vector_type(4)));
template <bool V4>
__global__ __launch_bounds__(kThreads) void bwd_sa_sig_kernel(const float* __restrict__ g,
                                                              const float* __restrict__ sa,
                                                              float* __restrict__ dz, int C, int HW) {
  // a block covers 4 * kThreads consecutive positions: V4, thread t the four at
  // 4 t (16-B loads); else the four at t + e kThreads (every load a 256-B segment)
  const int b = blockIdx.y;
  const int base = blockIdx.x * 4 * kThreads;
  const int Ch = C / 2;
  int pos[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) pos[e] = V4 ? base + 4 * threadIdx.x + e : base + threadIdx.x + e * kThreads;
  if (pos[0] >= HW) return;
  const float* gb = g + (size_t)b * C * HW;
  float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;   // four channels of each half in flight; each position sums in channel order
  if constexpr (V4) {
    const float* gp = gb + pos[0];
    int c = 0;
    for (; c + U <= Ch; c += U) {
      f32x4c v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v0[u] = *reinterpret_cast<const f32x4c*>(gp + (size_t)(c + u) * HW);
        v1[u] = *reinterpret_cast<const f32x4c*>(gp + (size_t)(Ch + c + u) * HW);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) { s0[e] += v0[u][e]; s1[e] += v1[u][e]; }
    }
    for (; c < Ch; ++c) {
      const f32x4c v0 = *reinterpret_cast<const f32x4c*>(gp + (size_t)c * HW);
      const f32x4c v1 = *reinterpret_cast<const f32x4c*>(gp + (size_t)(Ch + c) * HW);
#pragma unroll
      for (int e = 0; e < 4; ++e) { s0[e] += v0[e]; s1[e] += v1[e]; }
    }
  } else {
    int q[4];   // clamped positions: loads stay in range, results past HW are not stored
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = min(pos[e], HW - 1);
    int c = 0;
    for (; c + U <= Ch; c += U) {
      float v0[U][4], v1[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[u][e] = gb[(size_t)(c + u) * HW + q[e]];
          v1[u][e] = gb[(size_t)(Ch + c + u) * HW + q[e]];
        }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) { s0[e] += v0[u][e]; s1[e] += v1[u][e]; }
    }
    for (; c < Ch; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) { s0[e] += gb[(size_t)c * HW + q[e]]; s1[e] += gb[(size_t)(Ch + c) * HW + q[e]]; }
  }
  const size_t o0 = ((size_t)b * 2) * HW, o1 = o0 + HW;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (pos[e] >= HW) continue;
    const float y0 = sa[o0 + pos[e]], y1 = sa[o1 + pos[e]];
    dz[o0 + pos[e]] = s0[e] * (1.f - y0) * y0;
    dz[o1 + pos[e]] = s1[e] * (1.f - y1) * y1;
  }
}

// dx = gx1 * ca + dmean/HW + [hw is the HW-argmax of (b, c)] * dmax
__global__ __launch_bounds__(kThreads) void bwd_dx_kernel(const float* __restrict__ g, const float* __restrict__ dP,
                                                          const short* __restrict__ idx, const float* __restrict__ ca,
                                                          const float* __restrict__ dmean, const float* __restrict__ dmax,
                                                          const int* __restrict__ amax, float* __restrict__ dx, int C,
                                                          int HW) {
  const int b = blockIdx.y;
  const int hw = blockIdx.x * kThreads + threadIdx.x;
  extern __shared__ float sh[];
  float* sca = sh;
  float* smean = sh + C;
  float* smax = sh + 2 * C;
  int* samax = reinterpret_cast<int*>(sh + 3 * C);
  const float invhw = 1.f / (float)HW;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const size_t o = (size_t)b * C + c;
    sca[c] = ca[o];
    smean[c] = dmean[o] * invhw;
    smax[c] = dmax[o];
    samax[c] = amax[o];
  }
  __syncthreads();
  if (hw >= HW) return;
  const int Ch = C / 2;
  const float inv = 1.f / (float)Ch;
  float pa[2], pm[2];
  int pi[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    pa[h] = dP[((size_t)b * 4 + 2 * h) * HW + hw] * inv;
    pm[h] = dP[((size_t)b * 4 + 2 * h + 1) * HW + hw];
    pi[h] = idx[((size_t)b * 2 + h) * HW + hw];
  }
  const size_t base = (size_t)b * C * HW + hw;
#pragma unroll 8
  for (int c = 0; c < C; ++c) {
    const int h = c < Ch ? 0 : 1, cc = c - h * Ch;
    const size_t o = base + (size_t)c * HW;
    const float gx = g[o] + pa[h] + (pi[h] == cc ? pm[h] : 0.f);
    dx[o] = gx * sca[c] + smean[c] + (samax[c] == hw ? smax[c] : 0.f);
  }
}

int check(int B, int C, int HW) {
  if (B <= 0 || C <= 0 || HW <= 0) return SE_E_ARG;
  if (C % 2 || C / 2 > 32767) return SE_E_SHAPE;
  if ((long long)B * C * HW >= (1ll << 40)) return SE_E_SHAPE;
  return SE_OK;
}

dim3 hw_grid(int B, int HW) { return dim3((HW + kThreads - 1) / kThreads, B); }
int dca_tiles(int HW) { return (HW + kPos * kThreads - 1) / (kPos * kThreads); }

}  // namespace

namespace {

// ---------------------------------------------------------------------------
// Channel-attention MLP (ccbam.py:28-63): the avg- and max-pooled descriptors p
// ([2B, C]: rows b < B = mean, rows B + b = max) through the shared
//   ComplexLinear(C, Hd, bias=False) -> ReLU -> ComplexLinear(Hd, C, bias=False)
// (complex_nn.py:93-113: the real half of a row through real_linear, the imaginary
// half through imag_linear, no cross terms), then ca = sigmoid(o_avg + o_max).
// One workgroup: the whole MLP is ~2B * C * Hd * 2 FMAs (FRCRN: 262 K), a few us,
// in place of ~10 ATen / rocBLAS launches forward and ~20 backward. Sums run in
// index order in fp32 (fp64 for the weight gradients over the 2B rows).
// w1r / w1i: [Hd/2][C/2], w2r / w2i: [C/2][Hd/2] (nn.Linear [out][in]).
constexpr int kMlpThreads = 256;
__device__ __forceinline__ float mlp_p(const float* mean, const float* mx, int B, int C, int r, int c) {
  return r < B ? mean[(long long)r * C + c] : mx[(long long)(r - B) * C + c];
}

__global__ void __launch_bounds__(kMlpThreads)
mlp_fwd_kernel(const float* __restrict__ mean, const float* __restrict__ mx, const float* __restrict__ w1r,
               const float* __restrict__ w1i, const float* __restrict__ w2r, const float* __restrict__ w2i,
               int B, int C, int Hd, float* __restrict__ ca, float* __restrict__ hsave) {
  extern __shared__ float sh[];   // h [2B][Hd]
  const int C2 = C / 2, H2 = Hd / 2;
  for (int idx = threadIdx.x; idx < 2 * B * Hd; idx += kMlpThreads) {
    const int r = idx / Hd, j = idx - r * Hd;
    const int half = j >= H2, jj = j - half * H2;
    const float* w = (half ? w1i : w1r) + (long long)jj * C2;
    float s = 0.f;
    for (int c = 0; c < C2; ++c) s = fmaf(w[c], mlp_p(mean, mx, B, C, r, half * C2 + c), s);
    s = fmaxf(s, 0.f);
    sh[idx] = s;
    hsave[idx] = s;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < B * C; idx += kMlpThreads) {
    const int b = idx / C, c = idx - b * C;
    const int half = c >= C2, cc = c - half * C2;
    const float* w = (half ? w2i : w2r) + (long long)cc * H2;
    const float* ha = sh + (long long)b * Hd + half * H2;
    const float* hm = sh + (long long)(B + b) * Hd + half * H2;
    float oa = 0.f, om = 0.f;
    for (int j = 0; j < H2; ++j) { oa = fmaf(w[j], ha[j], oa); om = fmaf(w[j], hm[j], om); }
    ca[idx] = 1.f / (1.f + expf(-(oa + om)));
  }
}

// Backward from dca [B, C]: dmean, dmax [B, C] and the four weight gradients.
__global__ void __launch_bounds__(kMlpThreads)
mlp_bwd_kernel(const float* __restrict__ dca, const float* __restrict__ ca, const float* __restrict__ mean,
               const float* __restrict__ mx, const float* __restrict__ hsave, const float* __restrict__ w1r,
               const float* __restrict__ w1i, const float* __restrict__ w2r, const float* __restrict__ w2i,
               int B, int C, int Hd, float* __restrict__ dmean, float* __restrict__ dmx, float* __restrict__ dw1r,
               float* __restrict__ dw1i, float* __restrict__ dw2r, float* __restrict__ dw2i) {
  extern __shared__ float sh[];   // g [B][C] (= dL/do of both the avg and the max row), dh [2B][Hd]
  float* g = sh;
  float* dh = sh + (long long)B * C;
  const int C2 = C / 2, H2 = Hd / 2;
  for (int idx = threadIdx.x; idx < B * C; idx += kMlpThreads) {
    const float a = ca[idx];
    g[idx] = dca[idx] * a * (1.f - a);
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 2 * B * Hd; idx += kMlpThreads) {
    const int r = idx / Hd, j = idx - r * Hd;
    const int half = j >= H2, jj = j - half * H2;
    const float* w = half ? w2i : w2r;
    const float* gr = g + (long long)(r % B) * C + half * C2;
    float s = 0.f;
    for (int cc = 0; cc < C2; ++cc) s = fmaf(w[(long long)cc * H2 + jj], gr[cc], s);
    dh[idx] = hsave[idx] > 0.f ? s : 0.f;
  }
  __syncthreads();
  // dW2[c][j] = sum_r g[r mod B][c] h[r][j]
  for (int idx = threadIdx.x; idx < C * H2; idx += kMlpThreads) {
    const int c = idx / H2, jj = idx - c * H2;
    const int half = c >= C2, cc = c - half * C2;
    double s = 0.0;
    for (int r = 0; r < 2 * B; ++r) s += (double)g[(long long)(r % B) * C + c] * hsave[(long long)r * Hd + half * H2 + jj];
    (half ? dw2i : dw2r)[(long long)cc * H2 + jj] = (float)s;
  }
  // dW1[j][c] = sum_r dh[r][j] p[r][c]
  for (int idx = threadIdx.x; idx < Hd * C2; idx += kMlpThreads) {
    const int j = idx / C2, cc = idx - j * C2;
    const int half = j >= H2, jj = j - half * H2;
    double s = 0.0;
    for (int r = 0; r < 2 * B; ++r) s += (double)dh[(long long)r * Hd + j] * mlp_p(mean, mx, B, C, r, half * C2 + cc);
    (half ? dw1i : dw1r)[(long long)jj * C2 + cc] = (float)s;
  }
  // dp[r][c] = sum_j w1[j][c] dh[r][j]
  for (int idx = threadIdx.x; idx < 2 * B * C; idx += kMlpThreads) {
    const int r = idx / C, c = idx - r * C;
    const int half = c >= C2, cc = c - half * C2;
    const float* w = half ? w1i : w1r;
    const float* d = dh + (long long)r * Hd + half * H2;
    float s = 0.f;
    for (int jj = 0; jj < H2; ++jj) s = fmaf(w[(long long)jj * C2 + cc], d[jj], s);
    (r < B ? dmean : dmx)[(long long)(r % B) * C + c] = s;
  }
}

}  // namespace

static int mlp_check(int B, int C, int Hd) {
  if (B <= 0 || C <= 0 || Hd <= 0 || (C & 1) || (Hd & 1)) return SE_E_ARG;
  const size_t lds = ((size_t)B * C + 2 * (size_t)B * Hd) * sizeof(float);
  return lds <= 64 * 1024 ? SE_OK : SE_E_UNSUPPORTED;   // one workgroup's LDS
}

extern "C" int se_ccbam_mlp_fwd(const float* mean, const float* mx, const float* w1r, const float* w1i,
                                const float* w2r, const float* w2i, int B, int C, int Hd, float* ca, float* hsave,
                                void* stream) {
  if (int rc = mlp_check(B, C, Hd)) return rc;
  if (!mean || !mx || !w1r || !w1i || !w2r || !w2i || !ca || !hsave) return SE_E_ARG;
  hipLaunchKernelGGL(mlp_fwd_kernel, dim3(1), dim3(kMlpThreads), 2 * (size_t)B * Hd * sizeof(float),
                     se::as_stream(stream), mean, mx, w1r, w1i, w2r, w2i, B, C, Hd, ca, hsave);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_mlp_bwd(const float* dca, const float* ca, const float* mean, const float* mx,
                                const float* hsave, const float* w1r, const float* w1i, const float* w2r,
                                const float* w2i, int B, int C, int Hd, float* dmean, float* dmx, float* dw1r,
                                float* dw1i, float* dw2r, float* dw2i, void* stream) {
  if (int rc = mlp_check(B, C, Hd)) return rc;
  if (!dca || !ca || !mean || !mx || !hsave || !w1r || !w1i || !w2r || !w2i || !dmean || !dmx || !dw1r || !dw1i ||
      !dw2r || !dw2i)
    return SE_E_ARG;
  hipLaunchKernelGGL(mlp_bwd_kernel, dim3(1), dim3(kMlpThreads), ((size_t)B * C + 2 * (size_t)B * Hd) * sizeof(float),
                     se::as_stream(stream), dca, ca, mean, mx, hsave, w1r, w1i, w2r, w2i, B, C, Hd, dmean, dmx, dw1r,
                     dw1i, dw2r, dw2i);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" size_t se_ccbam_workspace_size(int B, int C, int HW) {
  if (check(B, C, HW)) return 0;
  return (size_t)B * dca_tiles(HW) * C * sizeof(float);
}

extern "C" int se_ccbam_channel_pool(const float* x, float* mean, float* mx, int* amax, int B, int C, int HW,
                                     void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!x || !mean || !mx || !amax) return SE_E_ARG;
  hipLaunchKernelGGL(channel_pool_kernel, dim3(B * C), dim3(kThreads), 0, se::as_stream(stream), x, mean, mx, amax, HW);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_spatial_pool(const float* x, const float* ca, float* pooled, short* idx, int B, int C, int HW,
                                     void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!x || !ca || !pooled || !idx) return SE_E_ARG;
  hipLaunchKernelGGL(spatial_pool_kernel, hw_grid(B, HW), dim3(kThreads), C * sizeof(float), se::as_stream(stream), x,
                     ca, pooled, idx, C, HW);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_apply(const float* x, const float* ca, const float* sa, float* out, int B, int C, int HW,
                              float* out_amax, void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!x || !ca || !sa || !out) return SE_E_ARG;
  if (out_amax && hipMemsetAsync(out_amax, 0, sizeof(float), se::as_stream(stream)) != hipSuccess) return SE_E_LAUNCH;
  hipLaunchKernelGGL(apply_kernel, hw_grid(B, HW), dim3(kThreads), C * sizeof(float), se::as_stream(stream), x, ca,
                     sa, out, C, HW, (unsigned*)out_amax);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_bwd_sa(const float* gout, float* dsa, int B, int C, int HW, void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!gout || !dsa) return SE_E_ARG;
  hipLaunchKernelGGL(bwd_sa_kernel, hw_grid(B, HW), dim3(kThreads), 0, se::as_stream(stream), gout, dsa, C, HW);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_bwd_sa_sigmoid(const float* gout, const float* sa, float* dz, int B, int C, int HW,
                                       void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!gout || !sa || !dz) return SE_E_ARG;
  const dim3 grid((HW + 4 * kThreads - 1) / (4 * kThreads), B);
  if (HW % 4 == 0 && ((uintptr_t)gout & 15) == 0)
    hipLaunchKernelGGL(bwd_sa_sig_kernel<true>, grid, dim3(kThreads), 0, se::as_stream(stream), gout, sa, dz, C, HW);
  else
    hipLaunchKernelGGL(bwd_sa_sig_kernel<false>, grid, dim3(kThreads), 0, se::as_stream(stream), gout, sa, dz, C,
                       HW);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_bwd_dca(const float* gout, const float* x, const float* dpooled, const short* idx, float* dca,
                                int B, int C, int HW, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!gout || !x || !dpooled || !idx || !dca || !ws) return SE_E_ARG;
  if (ws_bytes < se_ccbam_workspace_size(B, C, HW)) return SE_E_WORKSPACE;
  const int nt = dca_tiles(HW);
  float* part = static_cast<float*>(ws);
  if ((C / 2) % 8 == 0)
    hipLaunchKernelGGL(bwd_dca_kernel<8>, dim3(nt, C / 8, B), dim3(kThreads), 0, se::as_stream(stream), gout, x, dpooled,
                       idx, part, C, HW, nt);
  else
    hipLaunchKernelGGL(bwd_dca_kernel<1>, dim3(nt, C, B), dim3(kThreads), 0, se::as_stream(stream), gout, x, dpooled, idx,
                       part, C, HW, nt);
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(dca_reduce_kernel, dim3((B * C + 255) / 256), dim3(256), 0, se::as_stream(stream), part, dca, B, C,
                     nt);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_ccbam_bwd_dx(const float* gout, const float* dpooled, const short* idx, const float* ca,
                               const float* dmean, const float* dmax, const int* amax, float* dx, int B, int C, int HW,
                               void* stream) {
  if (int rc = check(B, C, HW)) return rc;
  if (!gout || !dpooled || !idx || !ca || !dmean || !dmax || !amax || !dx) return SE_E_ARG;
  hipLaunchKernelGGL(bwd_dx_kernel, hw_grid(B, HW), dim3(kThreads), 4 * C * sizeof(float), se::as_stream(stream), gout,
                     dpooled, idx, ca, dmean, dmax, amax, dx, C, HW);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
