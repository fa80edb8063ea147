// Persistent single-layer LSTM recurrence (forward + BPTT) for the
// ComplexLSTM of FRCRN / DCCRN (reference: models/modules/complex_nn.py:115-145,
// which runs torch.nn.LSTM; gate order i, f, g, o; h0 = c0 = 0).
//
// The input projection X·W_ihᵀ + b_ih + b_hh and all weight gradients are
// plain GEMMs (se_gemm, csrc/gemm.hip). What remains is the strictly
// sequential part, which MIOpen runs as 2-3 launches per time step:
//
//   fwd:  z_t = xproj_t + W_hh h_{t-1};  i,f,o = σ(z), g = tanh(z)
//         c_t = f c_{t-1} + i g;  h_t = o tanh(c_t)
//   bwd:  dgates_t from (dy_t + W_hhᵀ dgates_{t+1}) and the saved gates / cells.
//
// One launch runs every time step. Each workgroup owns BS sequences of one
// stacked LSTM and ALL of W_hh (4H x H fp32 = 256 KB at H = 128) in VGPRs —
// thread r holds gate row r (fwd) or a 128-row slice of column k (bwd) — so
// workgroups never talk to each other; the recurrent operand goes through LDS
// (below). Per step and workgroup that is BS·4H·H MACs in 2·H packed FMAs per
// thread.
#include "common.hpp"

#include <cstdlib>


namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

// Branch-free tanh (ocml's tanhf branches, which splits the step loop into
// many basic blocks and defeats the unrolled step schedule). |x| < 1/16:
// odd Taylor series to x^7 (truncation < 1e-11 rel); else (1-e)/(1+e) with
// e = exp(-2|x|) (rel. error ~5e-7 from rounding of e).
__device__ __forceinline__ float tanh_bf(float x) {
  const float ax = fabsf(x), x2 = x * x;
  const float e = expf(-2.f * ax);
  const float big = copysignf((1.f - e) / (1.f + e), x);
  const float small = x * (1.f + x2 * (-1.f / 3.f + x2 * (2.f / 15.f + x2 * (-17.f / 315.f))));
  return ax < 0.0625f ? small : big;
}

struct LstmArgs {
  const float* xproj;   // [L] x [B*T rows] x (4H), row stride x_row, lstm stride x_lstm (elements)
  const float* w_hh;    // [L][4H][H]
  const float* dy;      // bwd: [L][B][T][H]
  const float* zero;    // fwd: >= H zero floats (h_{-1})
  float* h;             // [L][B][T][H]
  float* c;             // [L][B][T][H]
  float* gates;         // [L][B][T][4H]  post-activation i, f, g, o
  float* dgates;        // bwd: [L][B][T][4H] pre-activation gradients
  long long x_lstm;
  int x_row;
  int B, T;
  unsigned rev_mask;    // bit l: LSTM l runs right-to-left (bidirectional reverse direction)
};

// ---------------------------------------------------------------------------
// LDS exchange: the recurrent operand (h_{t-1} forward, dgates_t backward)
// never leaves the workgroup, so it goes through LDS: written by the cell
// update, one barrier, then read by every lane as 16-B broadcast loads (all
// lanes of a wave read the same address: no bank conflict) straight into the
// packed FMAs. No global round trip and no wait for the step's stores in the
// recurrence (they are only for the backward / the weight gradients). Round 2
// replaced a form that stored the operand and read it back with scalar loads
// as SGPR operands of v_pk_fma_f32 (fwd / bwd 1060 / 987 us vs 733 / 736 us per
// launch at FRCRN size, bit-identical: the same products in the same order).
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

// acc0 / acc1 += w[q] * (v[2q], v[2q+1]) for q even / odd, v = the H floats at
// src (LDS), read as 16-B broadcast loads (every lane the same address).
// Measured alternatives (FRCRN size, isolated, fwd / bwd per launch): v_readlane
// into SGPR operands 939 / 837 us; a k-split matvec (4 rows x 32 columns per
// lane, a quarter of the LDS->VGPR traffic) 696 us fwd; whole cells per wave
// (gates met by shuffles, one barrier per step) 805 us fwd; this form 733 / 736.
template <int H>
__device__ __forceinline__ void matvec_step(const f32x2 (&w)[H / 2], const float* src, f32x2& acc0, f32x2& acc1) {
  const f32x4* hv = reinterpret_cast<const f32x4*>(src);
#pragma unroll
  for (int c0 = 0; c0 < H / 4; c0 += 8) {   // chunks of 8 loads: bounded live registers
#pragma unroll
    for (int q4 = c0; q4 < c0 + 8; ++q4) {
      const f32x4 v = hv[q4];
      acc0 = __builtin_elementwise_fma(w[2 * q4], f32x2{v.x, v.y}, acc0);
      acc1 = __builtin_elementwise_fma(w[2 * q4 + 1], f32x2{v.z, v.w}, acc1);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int H, int BS>
__global__ __launch_bounds__(4 * H) void lstm_fwd_lds_kernel(LstmArgs a) {
  constexpr int G = 4 * H;
  const int r = threadIdx.x;
  const int l = blockIdx.y, b0 = blockIdx.x * BS;
  const bool rev = (a.rev_mask >> l) & 1u;
  const int T = a.T;

  f32x2 w[H / 2];
  {
    const f32x2* W = reinterpret_cast<const f32x2*>(a.w_hh + ((size_t)l * G + r) * H);
#pragma unroll
    for (int q = 0; q < H / 2; ++q) w[q] = W[q];
  }
  __shared__ float sg[BS][G];
  __shared__ __attribute__((aligned(16))) float sh[BS][H];   // h_{t-1}
  for (int i = r; i < BS * H; i += G) (&sh[0][0])[i] = 0.f;   // h_{-1} = 0

  const float* xp = a.xproj + (size_t)l * a.x_lstm + r;
  int brow[BS];
#pragma unroll
  for (int b = 0; b < BS; ++b) brow[b] = min(b0 + b, a.B - 1);
  const int gate = __builtin_amdgcn_readfirstlane(r / H);
  static_assert((4 * H) % (BS * H) == 0, "threads must cover the cells");
  const int cb = (r % (BS * H)) / H, cj = r % H;
  const size_t crow = (size_t)l * a.B + brow[cb];
  float cst = 0.f;
  const int dir = rev ? -1 : 1, t0 = rev ? T - 1 : 0;
  auto xload = [&](int sx, float* dst) __attribute__((always_inline)) {
    const float* q = xp + (size_t)(t0 + dir * min(sx, T - 1)) * a.x_row;
#pragma unroll
    for (int b = 0; b < BS; ++b) dst[b] = q[(size_t)brow[b] * T * a.x_row];
  };
  float xa[BS], xb[BS];
  xload(0, xa);
  xload(1, xb);
  __syncthreads();
  auto step = [&](int s, float* xs) __attribute__((always_inline)) {
    const int t = t0 + dir * s;
    float z[BS];
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      f32x2 acc0 = f32x2{0.f, 0.f}, acc1 = f32x2{0.f, 0.f};
      matvec_step<H>(w, &sh[b][0], acc0, acc1);
      z[b] = xs[b] + ((acc0.x + acc0.y) + (acc1.x + acc1.y));
    }
    float v[BS];
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      const float th = tanh_bf(z[b]), sg_ = sigmoidf(z[b]);
      v[b] = gate == 2 ? th : sg_;
      sg[b][r] = v[b];
    }
#pragma unroll
    for (int b = BS - 1; b >= 0; --b) a.gates[(((size_t)l * a.B + brow[b]) * T + t) * G + r] = v[b];
    __syncthreads();   // gates of the step complete; every read of h_{t-1} done
    {
      const float ig = sg[cb][cj], fg = sg[cb][H + cj], gg = sg[cb][2 * H + cj], og = sg[cb][3 * H + cj];
      cst = fg * cst + ig * gg;
      const float hv = og * tanh_bf(cst);
      const size_t o = (crow * T + t) * H + cj;
      a.c[o] = cst;
      a.h[o] = hv;
      sh[cb][cj] = hv;   // duplicate cells store the same value
    }
    xload(s + 2, xs);
    __syncthreads();   // h_t in LDS for the next step
  };
  int s = 0;
  for (; s + 1 < T; s += 2) {
    step(s, xa);
    step(s + 1, xb);
  }
  if (s < T) step(s, xa);
}

template <int H, int BS>
__global__ __launch_bounds__(4 * H) void lstm_bwd_lds_kernel(LstmArgs a) {
  constexpr int G = 4 * H;
  const int tid = threadIdx.x;
  const int k = tid % H;
  const int rq = __builtin_amdgcn_readfirstlane(tid / H);
  const int l = blockIdx.y, b0 = blockIdx.x * BS;
  const bool rev = (a.rev_mask >> l) & 1u;
  const int T = a.T;

  f32x2 w[H / 2];
  {
    const float* W = a.w_hh + ((size_t)l * G + rq * H) * H + k;
#pragma unroll
    for (int p = 0; p < H / 2; ++p) w[p] = f32x2{W[(2 * p) * H], W[(2 * p + 1) * H]};
  }
  __shared__ float sp[4][BS][H];
  __shared__ __attribute__((aligned(16))) float sdg[BS][G];   // dgates_t

  static_assert((4 * H) % (BS * H) == 0, "threads must cover the cells");
  const int cb = (tid % (BS * H)) / H, cj = tid % H;
  float dc = 0.f, dh_rec = 0.f;
  const size_t rowc = ((size_t)l * a.B + min(b0 + cb, a.B - 1)) * T;
  const int dir = rev ? -1 : 1, t0 = rev ? T - 1 : 0;

  struct Pre { float dy, c, cp, g[4]; };
  auto fetch = [&](int sx, Pre& p) __attribute__((always_inline)) {
    sx = max(sx, 0);
    const int t = t0 + dir * sx;
    const int tp = t0 + dir * max(sx - 1, 0);
    const size_t o = (rowc + t) * H + cj;
    p.dy = a.dy[o];
    p.c = a.c[o];
    p.cp = a.c[(rowc + tp) * H + cj] * (sx > 0 ? 1.f : 0.f);
    const float* gp = a.gates + (rowc + t) * G + cj;
#pragma unroll
    for (int q = 0; q < 4; ++q) p.g[q] = gp[q * H];
  };
  Pre pa, pb;
  fetch(T - 1, pa);
  fetch(T - 2, pb);

  auto cell_step = [&](int s, const Pre& pc_) __attribute__((always_inline)) {
    const int t = t0 + dir * s;
    const float dh = pc_.dy + dh_rec, ct = pc_.c, cp = pc_.cp;
    const float ig = pc_.g[0], fg = pc_.g[1], gg = pc_.g[2], og = pc_.g[3];
    const float tc = tanh_bf(ct);
    dc += dh * og * (1.f - tc * tc);
    const float d0 = dc * gg * ig * (1.f - ig);
    const float d1 = dc * cp * fg * (1.f - fg);
    const float d2 = dc * ig * (1.f - gg * gg);
    const float d3 = dh * tc * og * (1.f - og);
    dc *= fg;
    float* dg = a.dgates + (rowc + t) * G + cj;
    dg[0] = d0;
    dg[H] = d1;
    dg[2 * H] = d2;
    dg[3 * H] = d3;
    sdg[cb][cj] = d0;
    sdg[cb][H + cj] = d1;
    sdg[cb][2 * H + cj] = d2;
    sdg[cb][3 * H + cj] = d3;
  };
  auto rec_step = [&](int s, Pre& pc_) __attribute__((always_inline)) {
    fetch(s - 2, pc_);
    __syncthreads();   // dgates_t in LDS
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      f32x2 acc0 = f32x2{0.f, 0.f}, acc1 = f32x2{0.f, 0.f};
      matvec_step<H>(w, &sdg[b][rq * H], acc0, acc1);
      sp[rq][b][k] = (acc0.x + acc0.y) + (acc1.x + acc1.y);
    }
    __syncthreads();
    dh_rec = (sp[0][cb][cj] + sp[1][cb][cj]) + (sp[2][cb][cj] + sp[3][cb][cj]);
  };
  int s = T - 1;
  for (; s >= 2; s -= 2) {
    cell_step(s, pa);
    rec_step(s, pa);
    cell_step(s - 1, pb);
    rec_step(s - 1, pb);
  }
  if (s == 1) {
    cell_step(1, pa);
    rec_step(1, pa);
    cell_step(0, pb);
  } else {
    cell_step(0, pa);
  }
}

// sequences per workgroup, forward / backward (SE_LSTM_BS / SE_LSTM_BS_BWD, build-time): the
// backward at one (every CU busy, 1.82 -> 1.32 us per step alone; FRCRN step 97.7 -> 97.4 ms,
// same box, round 5), the forward at two (one was slower)
#ifndef SE_LSTM_BS
#define SE_LSTM_BS 2
#endif
#ifndef SE_LSTM_BS_BWD
#define SE_LSTM_BS_BWD 1
#endif
constexpr int kBS = SE_LSTM_BS, kBSB = SE_LSTM_BS_BWD;

template <int H>
int launch(bool bwd, const LstmArgs& a, int L, hipStream_t st) {
  if (bwd)
    hipLaunchKernelGGL((lstm_bwd_lds_kernel<H, kBSB>), dim3((a.B + kBSB - 1) / kBSB, L), dim3(4 * H), 0, st, a);
  else
    hipLaunchKernelGGL((lstm_fwd_lds_kernel<H, kBS>), dim3((a.B + kBS - 1) / kBS, L), dim3(4 * H), 0, st, a);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

int check(int L, int B, int T, int H) {
  if (L <= 0 || L > 32 || B <= 0 || T <= 0) return SE_E_ARG;
  if (H != 64 && H != 128) return SE_E_UNSUPPORTED;
  if ((long long)L * B * T * 4 * H >= (1ll << 40)) return SE_E_SHAPE;
  return SE_OK;
}

}  // namespace

extern "C" int se_lstm_supported(int hidden) { return hidden == 64 || hidden == 128; }

extern "C" int se_lstm_fwd(const float* xproj, long long x_lstm_stride, int x_row_stride, const float* w_hh,
                           const float* zero, float* h, float* c, float* gates, int L, int B, int T, int H, unsigned rev_mask,
                           void* stream) {
  int rc = check(L, B, T, H);
  if (rc) return rc;
  if (x_row_stride < 4 * H) return SE_E_ARG;
  if (!xproj || !w_hh || !h || !c || !gates) return SE_E_ARG;
  if (!zero) return SE_E_ARG;
  LstmArgs a{xproj, w_hh, nullptr, zero, h, c, gates, nullptr, x_lstm_stride, x_row_stride, B, T, rev_mask};
  return H == 64 ? launch<64>(false, a, L, se::as_stream(stream)) : launch<128>(false, a, L, se::as_stream(stream));
}

extern "C" int se_lstm_bwd(const float* dy, const float* w_hh, const float* gates, const float* c,
                           float* dgates, int L, int B, int T, int H, unsigned rev_mask, void* stream) {
  int rc = check(L, B, T, H);
  if (rc) return rc;
  if (!dy || !w_hh || !gates || !c || !dgates) return SE_E_ARG;
  LstmArgs a{nullptr, w_hh, dy, nullptr, nullptr, const_cast<float*>(c), const_cast<float*>(gates), dgates, 0, 0, B, T,
             rev_mask};
  return H == 64 ? launch<64>(true, a, L, se::as_stream(stream)) : launch<128>(true, a, L, se::as_stream(stream));
}
