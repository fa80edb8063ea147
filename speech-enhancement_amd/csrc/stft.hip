// ConvSTFT / ConviSTFT (models/conv_stft.py) as packed real FFTs in LDS.
//
// The reference implements the STFT as conv1d against a [N+2, 1, win] basis
// (conv_stft.py:56) and the inverse as conv_transpose1d against the pinv of
// that basis followed by a window^2 overlap-add normaliser (:101-106). Both
// are linear maps we evaluate with FFTs instead (O(N log N) per frame, HBM-
// bound), two real frames packed into one complex FFT of length N = nfft:
//
//   analysis  X[k]  = sum_{n<win} w[n] x[t*hop + n - pad] e^{-2 pi i k n / N}
//   synthesis the pinv basis is M (M^T M)^{-1} with M^T M = (N/2) I + ee^T + oo^T
//             (e, o = even / odd index indicators over n < win), so a frame is
//             w[n] * (z[n] - e/o correction)/(N/2) where
//             z[n] = Re sum_{k<=N/2} X[k] e^{+2 pi i k n / N}.
//
// Frames are gathered with the reflect pad folded into the load; the inverse
// is tiled over OUTPUT samples (halo frames recomputed) so every output sample
// is written exactly once, coalesced, with no atomics and no frame buffer.
#include "common.hpp"

#include <cstdlib>

#include <algorithm>
#include <cmath>


namespace {

constexpr int kThreads = 256;
constexpr int kMaxPasses = 12;
constexpr int kLdsBudget = 80 * 1024;

struct FftPlan {
  int N, npass;
  int radix[kMaxPasses];
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// -i * a
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }

// Stockham autosort FFT (forward sign) of P length-N sequences held in LDS.
// Returns the buffer that holds the result.
__device__ float2* fft_forward(float2* a, float2* b, int P, const FftPlan& pl, const float2* __restrict__ tw) {
  const int N = pl.N;
  int Ns = 1;
  for (int ps = 0; ps < pl.npass; ++ps) {
    const int R = pl.radix[ps];
    const int nbf = N / R;
    const int tstep = N / (Ns * R);
    for (int idx = threadIdx.x; idx < P * nbf; idx += blockDim.x) {
      const int pr = idx / nbf, j = idx - pr * nbf;
      const float2* src = a + pr * N;
      float2* dst = b + pr * N;
      const int k = j % Ns;
      float2 v[5];
      for (int q = 0; q < R; ++q) v[q] = src[j + q * nbf];
      if (Ns > 1)
        for (int q = 1; q < R; ++q) v[q] = cmul(v[q], tw[q * k * tstep]);  // < N
      const int d = (j / Ns) * Ns * R + k;
      if (R == 2) {
        dst[d] = cadd(v[0], v[1]);
        dst[d + Ns] = csub(v[0], v[1]);
      } else if (R == 4) {
        const float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
        const float2 t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
        dst[d] = cadd(t0, t2);
        dst[d + Ns] = cadd(t1, t3);
        dst[d + 2 * Ns] = csub(t0, t2);
        dst[d + 3 * Ns] = csub(t1, t3);
      } else if (R == 3) {
        const float h = 0.86602540378443864676f;
        const float2 s = cadd(v[1], v[2]), df = csub(v[1], v[2]);
        const float2 m = csub(v[0], cscale(s, 0.5f));
        const float2 r = cscale(mul_mi(df), h);
        dst[d] = cadd(v[0], s);
        dst[d + Ns] = cadd(m, r);
        dst[d + 2 * Ns] = csub(m, r);
      } else {  // R == 5
        const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
        const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
        const float2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
        const float2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
        const float2 a1 = cadd(v[0], cadd(cscale(t1, c1), cscale(t2, c2)));
        const float2 a2 = cadd(v[0], cadd(cscale(t1, c2), cscale(t2, c1)));
        const float2 b1 = mul_mi(cadd(cscale(t3, s1), cscale(t4, s2)));
        const float2 b2 = mul_mi(csub(cscale(t3, s2), cscale(t4, s1)));
        dst[d] = cadd(v[0], cadd(t1, t2));
        dst[d + Ns] = cadd(a1, b1);
        dst[d + 4 * Ns] = csub(a1, b1);
        dst[d + 2 * Ns] = cadd(a2, b2);
        dst[d + 3 * Ns] = csub(a2, b2);
      }
    }
    __syncthreads();
    float2* t = a; a = b; b = t;
    Ns *= R;
  }
  return a;
}

// Compile-time plan for the common nfft values: every pass's radix, stride and
// butterfly count are constants, so the index divisions become multiply-shifts
// and the pass loop unrolls (the runtime plan above serves any other nfft).
struct CPlan {
  int npass;
  int radix[kMaxPasses];
};
// Radix 8 and 10 first (640 = 8*8*10, 512 = 8*8*8, 400 = 8*10*5, 320 = 8*8*5,
// 256 = 8*8*4): three barrier-separated passes instead of five for nfft 640.
constexpr CPlan make_cplan(int N) {
  CPlan p{};
  int n = N;
  const int order[6] = {8, 10, 4, 2, 3, 5};
  for (int oi = 0; oi < 6; ++oi)
    while (n > 1 && n % order[oi] == 0 && p.npass < kMaxPasses) { p.radix[p.npass++] = order[oi]; n /= order[oi]; }
  return p;
}
constexpr int kMaxRadix = 10;

// 5-point DFT of (a0..a4) -> (x0..x4) (forward sign)
__device__ __forceinline__ void dft5(float2 a0, float2 a1, float2 a2, float2 a3, float2 a4, float2 (&x)[5]) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  const float2 t1 = cadd(a1, a4), t2 = cadd(a2, a3);
  const float2 t3 = csub(a1, a4), t4 = csub(a2, a3);
  const float2 p1 = cadd(a0, cadd(cscale(t1, c1), cscale(t2, c2)));
  const float2 p2 = cadd(a0, cadd(cscale(t1, c2), cscale(t2, c1)));
  const float2 q1 = mul_mi(cadd(cscale(t3, s1), cscale(t4, s2)));
  const float2 q2 = mul_mi(csub(cscale(t3, s2), cscale(t4, s1)));
  x[0] = cadd(a0, cadd(t1, t2));
  x[1] = cadd(p1, q1);
  x[4] = csub(p1, q1);
  x[2] = cadd(p2, q2);
  x[3] = csub(p2, q2);
}

template <int R>
__device__ __forceinline__ void butterfly(float2 (&v)[kMaxRadix], float2* dst, int d, int Ns) {
  if constexpr (R == 8) {
    // X_k = E_k + W8^k O_k, X_{k+4} = E_k - W8^k O_k (E, O: 4-point DFTs of even / odd inputs)
    const float r = 0.70710678118654752440f;
    const float2 a0 = cadd(v[0], v[4]), a1 = csub(v[0], v[4]);
    const float2 a2 = cadd(v[2], v[6]), a3 = mul_mi(csub(v[2], v[6]));
    const float2 a4 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
    const float2 a6 = cadd(v[3], v[7]), a7 = mul_mi(csub(v[3], v[7]));
    const float2 e0 = cadd(a0, a2), e2 = csub(a0, a2), e1 = cadd(a1, a3), e3 = csub(a1, a3);
    const float2 o0 = cadd(a4, a6), o2 = csub(a4, a6), o1 = cadd(a5, a7), o3 = csub(a5, a7);
    const float2 w1 = make_float2(r * (o1.x + o1.y), r * (o1.y - o1.x));     // W8^1 o1, W8 = (1 - i)/sqrt2
    const float2 w2 = mul_mi(o2);                                            // W8^2 = -i
    const float2 w3 = make_float2(r * (o3.y - o3.x), -r * (o3.x + o3.y));    // W8^3 = (-1 - i)/sqrt2
    dst[d] = cadd(e0, o0);
    dst[d + 4 * Ns] = csub(e0, o0);
    dst[d + Ns] = cadd(e1, w1);
    dst[d + 5 * Ns] = csub(e1, w1);
    dst[d + 2 * Ns] = cadd(e2, w2);
    dst[d + 6 * Ns] = csub(e2, w2);
    dst[d + 3 * Ns] = cadd(e3, w3);
    dst[d + 7 * Ns] = csub(e3, w3);
  } else if constexpr (R == 10) {
    // X_k = E_{k mod 5} + W10^k O_{k mod 5} (E, O: 5-point DFTs of even / odd inputs);
    // W10^5 = -1, so X_{k+5} = E_k - W10^k O_k
    float2 E[5], O[5];
    dft5(v[0], v[2], v[4], v[6], v[8], E);
    dft5(v[1], v[3], v[5], v[7], v[9], O);
    const float2 W[5] = {make_float2(1.f, 0.f),
                         make_float2(0.80901699437494742410f, -0.58778525229247312917f),
                         make_float2(0.30901699437494742410f, -0.95105651629515357212f),
                         make_float2(-0.30901699437494742410f, -0.95105651629515357212f),
                         make_float2(-0.80901699437494742410f, -0.58778525229247312917f)};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float2 t = k ? cmul(O[k], W[k]) : O[0];
      dst[d + k * Ns] = cadd(E[k], t);
      dst[d + (k + 5) * Ns] = csub(E[k], t);
    }
  } else if constexpr (R == 2) {
    dst[d] = cadd(v[0], v[1]);
    dst[d + Ns] = csub(v[0], v[1]);
  } else if constexpr (R == 4) {
    const float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const float2 t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
    dst[d] = cadd(t0, t2);
    dst[d + Ns] = cadd(t1, t3);
    dst[d + 2 * Ns] = csub(t0, t2);
    dst[d + 3 * Ns] = csub(t1, t3);
  } else if constexpr (R == 3) {
    const float h = 0.86602540378443864676f;
    const float2 s = cadd(v[1], v[2]), df = csub(v[1], v[2]);
    const float2 m = csub(v[0], cscale(s, 0.5f));
    const float2 r = cscale(mul_mi(df), h);
    dst[d] = cadd(v[0], s);
    dst[d + Ns] = cadd(m, r);
    dst[d + 2 * Ns] = csub(m, r);
  } else {
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const float2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
    const float2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
    const float2 a1 = cadd(v[0], cadd(cscale(t1, c1), cscale(t2, c2)));
    const float2 a2 = cadd(v[0], cadd(cscale(t1, c2), cscale(t2, c1)));
    const float2 b1 = mul_mi(cadd(cscale(t3, s1), cscale(t4, s2)));
    const float2 b2 = mul_mi(csub(cscale(t3, s2), cscale(t4, s1)));
    dst[d] = cadd(v[0], cadd(t1, t2));
    dst[d + Ns] = cadd(a1, b1);
    dst[d + 4 * Ns] = csub(a1, b1);
    dst[d + 2 * Ns] = cadd(a2, b2);
    dst[d + 3 * Ns] = csub(a2, b2);
  }
}

template <int N, int P, int PS, int NS>
__device__ float2* fft_pass(float2* a, float2* b, const float2* __restrict__ tw) {
  constexpr CPlan pl = make_cplan(N);
  if constexpr (PS == pl.npass) {
    return a;
  } else {
    constexpr int R = pl.radix[PS], nbf = N / R, tstep = N / (NS * R);
    for (int idx = threadIdx.x; idx < P * nbf; idx += kThreads) {
      const int pr = idx / nbf, j = idx - pr * nbf;
      const float2* src = a + pr * N;
      float2* dst = b + pr * N;
      const int k = j % NS;
      float2 v[kMaxRadix];
#pragma unroll
      for (int q = 0; q < R; ++q) v[q] = src[j + q * nbf];
      if constexpr (NS > 1) {
#pragma unroll
        for (int q = 1; q < R; ++q) v[q] = cmul(v[q], tw[q * k * tstep]);
      }
      butterfly<R>(v, dst, (j / NS) * NS * R + k, NS);
    }
    __syncthreads();
    return fft_pass<N, P, PS + 1, NS * R>(b, a, tw);
  }
}

// In-place variant of fft_pass: every thread first reads all its butterfly
// inputs of the pass into registers, then (after a barrier) writes all outputs
// into the SAME buffer. Half the LDS of the ping-pong form, so a block holds
// twice the frames (16 at nfft 640) and writes 64-B row segments.
template <int N, int P, int PS, int NS, int TPB = kThreads>
__device__ void fft_pass_ip(float2* a, const float2* __restrict__ tw) {
  constexpr CPlan pl = make_cplan(N);
  if constexpr (PS < pl.npass) {
    constexpr int R = pl.radix[PS], nbf = N / R, tstep = N / (NS * R);
    constexpr int ITER = (P * nbf + TPB - 1) / TPB;
    float2 v[ITER][kMaxRadix];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = threadIdx.x + it * TPB;
      if (P * nbf % TPB == 0 || idx < P * nbf) {
        const int pr = idx / nbf, j = idx - pr * nbf;
        const float2* src = a + pr * N;
        const int k = j % NS;
#pragma unroll
        for (int q = 0; q < R; ++q) v[it][q] = src[j + q * nbf];
        if constexpr (NS > 1) {
#pragma unroll
          for (int q = 1; q < R; ++q) v[it][q] = cmul(v[it][q], tw[q * k * tstep]);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = threadIdx.x + it * TPB;
      if (P * nbf % TPB == 0 || idx < P * nbf) {
        const int pr = idx / nbf, j = idx - pr * nbf;
        const int k = j % NS;
        butterfly<R>(v[it], a + pr * N, (j / NS) * NS * R + k, NS);
      }
    }
    __syncthreads();
    fft_pass_ip<N, P, PS + 1, NS * R, TPB>(a, tw);
  }
}

// FFT of P sequences: compile-time plan when CN != 0, else the runtime plan.
template <int CN, int CP>
__device__ __forceinline__ float2* fft_any(float2* a, float2* b, int P, const FftPlan& pl, const float2* tw) {
  if constexpr (CN != 0) {
    // twiddles staged in LDS once per block: every pass reads them inside its
    // barrier-separated loop, where a global (L2) read is latency on the
    // critical path
    __shared__ float2 stw[CN];
    for (int i = threadIdx.x; i < CN; i += kThreads) stw[i] = tw[i];
    __syncthreads();
    return fft_pass<CN, CP, 0, 1>(a, b, stw);
  } else {
    return fft_forward(a, b, P, pl, tw);
  }
}

// XCD-aware (frame block, utterance) of a (ceil(T / frames), B) grid: dispatch
// round-robins consecutive workgroups over the 8 XCDs, so the two blocks that
// write the 64-B halves of one 128-B spectrum row segment would sit on
// different XCDs and each L2 would write back a partial line. The bijective
// remap gives consecutive frame blocks of an utterance to one XCD, dispatched
// back to back, so the halves merge in that L2 before write-back.
__device__ __forceinline__ void xcd_frame_group(int L, int total, int nx, int& tb, int& b) {
  constexpr int kXcd = 8;
  const int xcd = L % kXcd, idx = L / kXcd;
  const int q = total / kXcd, r = total % kXcd;
  const int t = xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
  b = t / nx;
  tb = t - b * nx;
}
__device__ __forceinline__ void xcd_frame_block(int& tb, int& b) {
  xcd_frame_group(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, gridDim.x, tb, b);
}

// Storage type of the signal / spectrum tensors (SE_DTYPE_*). LP = false: fp32 (the
// kernels as they were); LP = true: bf16 or fp16 by the launch's dt (a uniform
// branch per access), converted to fp32 on load and rounded to nearest even on store.
template <bool LP>
__device__ __forceinline__ float ldx(const void* p, long long i, int dt) {
  if constexpr (!LP) return static_cast<const float*>(p)[i];
  else return dt == SE_DTYPE_BF16 ? (float)static_cast<const __bf16*>(p)[i] : (float)static_cast<const _Float16*>(p)[i];
}
template <bool LP>
__device__ __forceinline__ void stx(void* p, long long i, float v, int dt) {
  if constexpr (!LP) static_cast<float*>(p)[i] = v;
  else if (dt == SE_DTYPE_BF16) static_cast<__bf16*>(p)[i] = (__bf16)v;
  else static_cast<_Float16*>(p)[i] = (_Float16)v;
}

__device__ __forceinline__ int reflect_index(int i, int L) {
  if (i < 0) i = -i;
  if (i >= L) i = 2 * (L - 1) - i;
  return i;
}

__device__ __forceinline__ int floor_div(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }
// floor(a / d) for 0 <= a < 2^22 from a float reciprocal rd = 1 / d, corrected by one
// step either way (the product is off by less than one): a few VALU instead of the
// ~40 of an integer division, in the per-sample overlap-add loops
__device__ __forceinline__ int fdiv_nn(int a, int d, float rd) {
  int q = (int)((float)a * rd);
  q -= q * d > a ? 1 : 0;
  q += (q + 1) * d <= a ? 1 : 0;
  return q;
}
__device__ __forceinline__ int ceil_div_i(int a, int b) { return -floor_div(-a, b); }

// Unpack two packed real-FFT results (pair j) and store rows k = 0..N/2 of frames
// t0 + 2j, t0 + 2j + 1. out layout [B, N+2, T] or mags/phase [B, N/2+1, T].
template <int CN, int CP, bool LP = false>
__device__ void unpack_store(const float2* Z, int Pr, int Nr, int t0, int T, int b,
                             void* out0, void* out1, int mag_phase, int dt) {
  const int N = CN ? CN : Nr, P = CP ? CP : Pr;
  const int half = N / 2 + 1;
  const int FT = 2 * P;
  for (int idx = threadIdx.x; idx < half * FT; idx += blockDim.x) {
    const int k = idx / FT, f = idx - k * FT;
    const int t = t0 + f;
    if (t >= T) continue;
    const int j = f >> 1;
    const float2 zk = Z[j * N + k];
    const float2 zc = Z[j * N + ((N - k) % N)];
    float re, im;
    if ((f & 1) == 0) {  // (Z[k] + conj Z[N-k]) / 2
      re = 0.5f * (zk.x + zc.x);
      im = 0.5f * (zk.y - zc.y);
    } else {             // (Z[k] - conj Z[N-k]) / (2i)
      re = 0.5f * (zk.y + zc.y);
      im = -0.5f * (zk.x - zc.x);
    }
    im += 0.f;   // -0 -> +0: DC / Nyquist imag parts are exact zeros (atan2 branch cut)
    if (!mag_phase) {
      stx<LP>(out0, ((long long)b * (2 * half) + k) * T + t, re, dt);
      stx<LP>(out0, ((long long)b * (2 * half) + half + k) * T + t, im, dt);
    } else {
      stx<LP>(out0, ((long long)b * half + k) * T + t, sqrtf(re * re + im * im), dt);
      stx<LP>(out1, ((long long)b * half + k) * T + t, atan2f(im, re), dt);
    }
  }
}

struct StftArgs {
  const void* x;       // [B, L]
  void* out0;
  void* out1;
  int dt;              // SE_DTYPE_* of x / out0 / out1
  const float* window; // [win]
  const float2* tw;    // [N]
  int L, win, hop, T, pad, mag_phase, P;
  FftPlan pl;
};

// grid (ceil(T / 2P), B)
template <int CN, int CP, bool LP = false>
__global__ void __launch_bounds__(kThreads) stft_fwd_kernel(const StftArgs a) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const int N = CN ? CN : a.pl.N, P = CP ? CP : a.P;
  float2* A = lds;
  float2* Bf = lds + P * N;
  const int b = blockIdx.y, t0 = blockIdx.x * 2 * P;
  const long long xo = (long long)b * a.L;
  for (int idx = threadIdx.x; idx < P * N; idx += blockDim.x) {
    const int j = idx / N, n = idx - j * N;
    const int ta = t0 + 2 * j, tb = ta + 1;
    float ya = 0.f, yb = 0.f;
    if (n < a.win) {
      const float w = a.window[n];
      if (ta < a.T) ya = w * ldx<LP>(a.x, xo + reflect_index(ta * a.hop + n - a.pad, a.L), a.dt);
      if (tb < a.T) yb = w * ldx<LP>(a.x, xo + reflect_index(tb * a.hop + n - a.pad, a.L), a.dt);
    }
    A[idx] = make_float2(ya, yb);
  }
  __syncthreads();
  const float2* Z = fft_any<CN, CP>(A, Bf, P, a.pl, a.tw);
  unpack_store<CN, CP, LP>(Z, P, N, t0, a.T, b, a.out0, a.out1, a.mag_phase, a.dt);
}

// ConvSTFT with the in-place FFT: kPairsIP frame pairs per block in one LDS
// buffer (compiled plans only). grid (ceil(T / 2P), B)
// 4 pairs (8 frames, 25 KB of LDS, 6 blocks per CU) measured fastest at the FRCRN
// bench shape: 36.9 us per launch vs 46.9 (8 pairs), 40.0 (2), 89.8 (16)
// (tools/stft_micro.py; the XCD-aware block order merges the 32-B row segments
// of neighbouring blocks in one L2)
constexpr int kPairsIP = 4;
template <int CN, int P = kPairsIP, bool LP = false>
__global__ void __launch_bounds__(kThreads) stft_fwd_ip_kernel(const StftArgs a) {
  constexpr int TPB = kThreads;
  constexpr int N = CN;
  __shared__ __attribute__((aligned(16))) float2 A[P * N];
  __shared__ float2 stw[N];
  int tb, b;
  xcd_frame_block(tb, b);
  const int t0 = tb * 2 * P;
  const long long xo = (long long)b * a.L;
  for (int i = threadIdx.x; i < N; i += TPB) stw[i] = a.tw[i];
  // frame gather: all of a thread's loads are issued before any is used
  // (compile-time trip count; branch-free clamped addresses and zero weights),
  // so the block pays one memory latency instead of one per element
  constexpr int IT = (P * N + TPB - 1) / TPB;
  float ya[IT], yb[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * TPB;
    const int j = idx / N, n = idx - j * N;
    const int ta = t0 + 2 * j, tb = ta + 1;
    const bool ok = idx < P * N && n < a.win;
    const int nn = ok ? n : 0;
    const float w = ok ? a.window[nn] : 0.f;
    const float xa = ldx<LP>(a.x, xo + reflect_index(min(ta, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
    const float xb = ldx<LP>(a.x, xo + reflect_index(min(tb, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
    ya[it] = ta < a.T ? w * xa : 0.f;
    yb[it] = tb < a.T ? w * xb : 0.f;
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * TPB;
    if (idx < P * N) A[idx] = make_float2(ya[it], yb[it]);
  }
  __syncthreads();
  fft_pass_ip<N, P, 0, 1, TPB>(A, stw);
  unpack_store<CN, P, LP>(A, P, N, t0, a.T, b, a.out0, a.out1, a.mag_phase, a.dt);
}

// ---------------------------------------------------------------------------
// Wave-local forms: one frame pair per wave, its FFT passes synchronised by the
// wave's own in-order LDS traffic (no block barrier between passes), so every
// wave runs its load -> FFT chain independently and W of them share a block only
// for the coalesced spectrum store (2W frames per row segment, one barrier).

#ifndef SE_STFT_WV
#define SE_STFT_WV 1
#endif
// W pairs per block: 8 (16 frames, 64-B row segments, 45 KB of LDS at nfft 640)
#ifndef SE_STFT_WV_PAIRS
#define SE_STFT_WV_PAIRS 8
#endif
constexpr int kWvPairs = SE_STFT_WV_PAIRS;
// the register-radix ConvSTFT for nfft 640 / 512 / 320 (stft_fwd_rg_kernel); 0: the wave-local form
#ifndef SE_STFT_RG
#define SE_STFT_RG 1
#endif
using se::kWave;
// Twiddle table per wave-local kernel: staged in LDS (1) or read through L1 (0). The
// forward and the adjoint read it through L1 (the FFT passes' LDS traffic drops by the
// twiddle reads, and the forward's waves need no block barrier before their FFTs); the
// iSTFT forward, whose spectrum gather sweeps L1, stages it
#ifndef SE_STFT_TWL_FWD
#define SE_STFT_TWL_FWD 0
#endif
#ifndef SE_STFT_TWL_IFWD
#define SE_STFT_TWL_IFWD 1
#endif
#ifndef SE_STFT_TWL_IBWD
#define SE_STFT_TWL_IBWD 0
#endif


// compiler barrier between a wave's LDS writes and its reads of other lanes' data:
// LDS instructions of one wave execute in issue order, so only code motion must stop
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// In-place pass PS of the compiled plan over ONE sequence a[0..N) by one wave:
// every lane reads all inputs of its butterflies, then writes all outputs.
template <int N, int PS, int NS>
__device__ __forceinline__ void wfft_pass(float2* a, const float2* __restrict__ tw, int lane) {
  constexpr CPlan pl = make_cplan(N);
  if constexpr (PS < pl.npass) {
    constexpr int R = pl.radix[PS], nbf = N / R, tstep = N / (NS * R);
    constexpr int ITER = (nbf + kWave - 1) / kWave;
    float2 v[ITER][kMaxRadix];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int j = lane + it * kWave;
      if (nbf % kWave == 0 || j < nbf) {
        const int k = j % NS;
#pragma unroll
        for (int q = 0; q < R; ++q) v[it][q] = a[j + q * nbf];
        if constexpr (NS > 1) {
#pragma unroll
          for (int q = 1; q < R; ++q) v[it][q] = cmul(v[it][q], tw[q * k * tstep]);
        }
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int j = lane + it * kWave;
      if (nbf % kWave == 0 || j < nbf) butterfly<R>(v[it], a, (j / NS) * NS * R + j % NS, NS);
    }
    wave_lds_sync();
    wfft_pass<N, PS + 1, NS * R>(a, tw, lane);
  }
}


// Pair stride of the wave-local LDS image: N + 2 float2, so the unpack's reads of
// W pairs at one bin fall in different banks
template <int N> constexpr int wv_stride() { return N + 2; }
// frame pairs per block of the wave-local kernels (7 per block to fit four blocks per
// CU, and 4 or 16 per block, measured slower: profiles/ab/r4_stft_regs_pairs_ab.txt)
template <int N> constexpr int wv_pairs() { return kWvPairs; }

// Unpack the W packed pair results of a wave-local block (pair stride NP) into
// frames t0 + 2j (even) and t0 + 2j + 1 (odd); lanes run along frames, so a store
// covers 2W consecutive frames of a spectrum row. out layout [B, N+2, T], or
// mags / phase [B, N/2+1, T].
template <int N, int W, bool LP>
__device__ __forceinline__ void wv_unpack_store(const float2* A, int t0, int T, int b, void* out0, void* out1,
                                                int mag_phase, int dt) {
  constexpr int NP = wv_stride<N>(), TPB = kWave * W, half = N / 2 + 1, FT = 2 * W;
  // offsets from the utterance's rows (32-bit: (N + 2) T elements per utterance)
  const long long ub = (long long)b * (mag_phase ? half : 2 * half) * T;
  for (int idx = threadIdx.x; idx < half * FT; idx += TPB) {
    const int k = idx / FT, f = idx - k * FT;
    const int t = t0 + f;
    if (t >= T) continue;
    const int j = f >> 1;
    const float2 zk = A[j * NP + k];
    const float2 zc = A[j * NP + ((N - k) % N)];
    float re, im;
    if ((f & 1) == 0) {   // (Z[k] + conj Z[N-k]) / 2
      re = 0.5f * (zk.x + zc.x);
      im = 0.5f * (zk.y - zc.y);
    } else {              // (Z[k] - conj Z[N-k]) / (2i)
      re = 0.5f * (zk.y + zc.y);
      im = -0.5f * (zk.x - zc.x);
    }
    im += 0.f;   // -0 -> +0 (atan2 branch cut)
    const int o = k * T + t;
#if SE_RG_PROBE == 2   // probe: no spectrum stores (kept live by an impossible condition)
    if (re != 1234.5f) continue;
#endif
    if (!mag_phase) {
      if constexpr (!LP) {
        float* op = static_cast<float*>(out0) + ub;
        op[o] = re;
        op[o + half * T] = im;
      } else {
        stx<LP>(out0, ub + o, re, dt);
        stx<LP>(out0, ub + o + half * T, im, dt);
      }
    } else {
      stx<LP>(out0, ub + o, sqrtf(re * re + im * im), dt);
      stx<LP>(out1, ub + o, atan2f(im, re), dt);
    }
  }
}

// ConvSTFT, wave-local FFT: W frame pairs per block (wave w: frames t0 + 2w, +1).
// grid (ceil(T / 2W), B), 64 W threads
template <int CN, int W = wv_pairs<CN>(), bool LP = false>
__global__ void __launch_bounds__(kWave * W) stft_fwd_wv_kernel(const StftArgs a) {
  constexpr int N = CN, NP = wv_stride<N>(), TPB = kWave * W;
  constexpr int half = N / 2 + 1, FT = 2 * W;
  __shared__ __attribute__((aligned(16))) float2 A[W * NP];
#if SE_STFT_TWL_FWD
  __shared__ float2 stw[N];
#else
  const float2* stw = a.tw;
#endif
  int tb, b;
  xcd_frame_block(tb, b);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int t0 = tb * FT, ta = t0 + 2 * w, tbb = ta + 1;
  const long long xo = (long long)b * a.L;
  // the wave's two frames: loads for n < win only (the rest of the FFT input is
  // zero), all issued before any is used. Frames clear of both signal ends (all but
  // a few per utterance, wave-uniform) index the signal directly: 32-bit offsets from
  // the utterance's base, no reflect
  constexpr int IT = (N + kWave - 1) / kWave;
  float ya[IT], yb[IT];
  const int sa = ta * a.hop - a.pad;
  if (!LP && sa >= 0 && tbb < a.T && sa + a.hop + a.win <= a.L) {
    const float* xp = static_cast<const float*>(a.x) + xo + sa;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int n = lane + it * kWave;
      const bool ok = n < a.win;
      const int nn = ok ? n : 0;
      const float wv = ok ? a.window[nn] : 0.f;
      ya[it] = wv * xp[nn];
      yb[it] = wv * xp[a.hop + nn];
    }
  } else {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int n = lane + it * kWave;
      const bool ok = n < a.win;
      const int nn = ok ? n : 0;
      const float wv = ok ? a.window[nn] : 0.f;
      const float xa = ldx<LP>(a.x, xo + reflect_index(min(ta, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
      const float xb = ldx<LP>(a.x, xo + reflect_index(min(tbb, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
      ya[it] = ta < a.T ? wv * xa : 0.f;
      yb[it] = tbb < a.T ? wv * xb : 0.f;
    }
  }
#if SE_STFT_TWL_FWD
  for (int i = threadIdx.x; i < N; i += TPB) stw[i] = a.tw[i];
#endif
  float2* Aw = A + w * NP;
#if SE_STFT_TWL_FWD
  __syncthreads();   // stw
#endif
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int n = lane + it * kWave;
    if (N % kWave == 0 || n < N) Aw[n] = make_float2(ya[it], yb[it]);
  }
  wave_lds_sync();   // the wave's own pair only
  wfft_pass<N, 0, 1>(Aw, stw, lane);
  __syncthreads();   // every pair of the block transformed
  wv_unpack_store<N, W, LP>(A, t0, a.T, b, a.out0, a.out1, a.mag_phase, a.dt);
}

// ---------------------------------------------------------------------------
// Register-radix ConvSTFT (nfft = 64 R, R = 10 / 8 / 5: 640, 512, 320). One frame pair per
// wave, N = 64 x R as a two-level decomposition n = l + 64 q (lane l, register q):
//   1. the gather leaves each lane its R samples x[l + 64 q] in registers (with win <= N/2
//      the upper R/2 are the zero padding, compile-time zeros: HALF);
//   2. an R-point DFT over q in registers, times the twiddle W_N^(l k1)  (no LDS);
//   3. the R results go to LDS as R rows of 64 (row k1, column l; padded rows), and each
//      row's 64-point DFT over l runs as two radix-8 passes (wave-local, in place);
//   4. row k1, column k2 then holds X[k1 + R k2], which the block's unpack reads by that map.
// One LDS round trip fewer than the three-pass wave-local form (stft_fwd_wv_kernel), and the
// first radix stage skips the zero half of the padded frame.
template <int R>
__device__ __forceinline__ void rdft(const float2 (&v)[kMaxRadix], float2 (&o)[kMaxRadix]) {
  if constexpr (R == 10) {
    float2 E[5], O[5];
    dft5(v[0], v[2], v[4], v[6], v[8], E);
    dft5(v[1], v[3], v[5], v[7], v[9], O);
    const float2 W[5] = {make_float2(1.f, 0.f),
                         make_float2(0.80901699437494742410f, -0.58778525229247312917f),
                         make_float2(0.30901699437494742410f, -0.95105651629515357212f),
                         make_float2(-0.30901699437494742410f, -0.95105651629515357212f),
                         make_float2(-0.80901699437494742410f, -0.58778525229247312917f)};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float2 t = k ? cmul(O[k], W[k]) : O[0];
      o[k] = cadd(E[k], t);
      o[k + 5] = csub(E[k], t);
    }
  } else if constexpr (R == 8) {
    const float r = 0.70710678118654752440f;
    const float2 a0 = cadd(v[0], v[4]), a1 = csub(v[0], v[4]);
    const float2 a2 = cadd(v[2], v[6]), a3 = mul_mi(csub(v[2], v[6]));
    const float2 a4 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
    const float2 a6 = cadd(v[3], v[7]), a7 = mul_mi(csub(v[3], v[7]));
    const float2 e0 = cadd(a0, a2), e2 = csub(a0, a2), e1 = cadd(a1, a3), e3 = csub(a1, a3);
    const float2 o0 = cadd(a4, a6), o2 = csub(a4, a6), o1 = cadd(a5, a7), o3 = csub(a5, a7);
    const float2 w1 = make_float2(r * (o1.x + o1.y), r * (o1.y - o1.x));
    const float2 w2 = mul_mi(o2);
    const float2 w3 = make_float2(r * (o3.y - o3.x), -r * (o3.x + o3.y));
    o[0] = cadd(e0, o0); o[4] = csub(e0, o0);
    o[1] = cadd(e1, w1); o[5] = csub(e1, w1);
    o[2] = cadd(e2, w2); o[6] = csub(e2, w2);
    o[3] = cadd(e3, w3); o[7] = csub(e3, w3);
  } else {
    static_assert(R == 5, "register radix: 10, 8 or 5");
    float2 x5[5];
    dft5(v[0], v[1], v[2], v[3], v[4], x5);
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = x5[k];
  }
}

#ifndef SE_RG_ROW
#define SE_RG_ROW 72
#endif
#ifndef SE_RG_NT
#define SE_RG_NT 0   // non-temporal spectrum stores (variant builds)
#endif
#ifndef SE_RG_PROBE
#define SE_RG_PROBE 0   // timing probes of the register-radix ConvSTFT (variant builds only)
#endif
#ifndef SE_RG_W
#define SE_RG_W 8
#endif
#ifndef SE_ISTFT_BWD_RG
#define SE_ISTFT_BWD_RG 1   // register-radix iSTFT adjoint (istft_bwd_rg_kernel)
#endif
#ifndef SE_ISTFT_FWD_RG
#define SE_ISTFT_FWD_RG 0   // register-radix FFT in the iSTFT forward (istft_fwd_wv_kernel<.., RG>)
#endif
#ifndef SE_IRG_W
#define SE_IRG_W 4          // its frame pairs per block (8: 38.4 vs 37.2 us, profiles/ab/r6_istft_bwd_rg.log)
#endif
#ifndef SE_RG_PPW
#define SE_RG_PPW 1
#endif
constexpr int kRgRow = SE_RG_ROW;   // float2 per LDS row of 64 (+8 pad: the radix-8 reads of 4 rows x
                                    // 8 columns land on 32 distinct even banks)

// Position of element i (0..63) of a row in LDS: 8 columns of 9 (one pad per 8), so the
// stride-1 (i = j + 8 q, lanes along j) and the stride-8 (i = 8 j + q, lanes along j)
// accesses of the radix-8 passes both spread a 32-lane group over 32 distinct banks
// (row stride kRgRow = 72 = 8 x 9: 4 rows x 8 columns per group)
__device__ __forceinline__ int rg_pos(int i) { return (i & 7) + 9 * (i >> 3); }

// the 64-point DFTs of the R rows of one wave's image (in place, Stockham order):
// pass 0 (Ns = 1): reads i = j + 8 q, writes 8 j + q; pass 1 (Ns = 8, twiddles
// W64^(q j) = W_N^(R q j)): reads and writes j + 8 q
template <int R, int PS, int ROWS = R>
__device__ __forceinline__ void rg_row_pass(float2* a, const float2* __restrict__ tw, int lane) {
  constexpr int NB = 8 * ROWS, ITER = (NB + kWave - 1) / kWave;
  float2 v[ITER][kMaxRadix];
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int bi = lane + it * kWave;
    if (NB % kWave == 0 || bi < NB) {
      const int r = bi >> 3, j = bi & 7;
      const float2* row = a + r * kRgRow;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[it][q] = row[j + 9 * q];   // rg_pos(j + 8 q)
      if constexpr (PS == 1) {
#pragma unroll
        for (int q = 1; q < 8; ++q) v[it][q] = cmul(v[it][q], tw[R * q * j]);
      }
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int bi = lane + it * kWave;
    if (NB % kWave == 0 || bi < NB) {
      const int r = bi >> 3, j = bi & 7;
      float2 o[kMaxRadix];
      rdft<8>(v[it], o);
      float2* row = a + r * kRgRow;
#pragma unroll
      for (int q = 0; q < 8; ++q) row[PS == 0 ? q + 9 * j : j + 9 * q] = o[q];   // rg_pos(8 j + q) / (j + 8 q)
    }
  }
  wave_lds_sync();
}

// W pairs per block, TPB threads; lanes along frames: a store covers 2W consecutive frames of
// a spectrum row (the per-(bin, pair) form with both frames of a pair per item measured slower:
// its stores interleave at a 2-frame stride)
template <int N, int R, int W, int TPB, bool LP>
__device__ __forceinline__ void rg_unpack_store(const float2* A, int t0, int T, int b, void* out0, void* out1,
                                                int mag_phase, int dt) {
  constexpr int half = N / 2 + 1, FT = 2 * W, WS = R * kRgRow;
  const long long ub = (long long)b * (mag_phase ? half : 2 * half) * T;
  for (int idx = threadIdx.x; idx < half * FT; idx += TPB) {
    const int k = idx / FT, f = idx - k * FT;
    const int t = t0 + f;
    if (t >= T) continue;
    const int j = f >> 1;
    const int kc = k ? N - k : 0;
    const float2 zk = A[j * WS + (k % R) * kRgRow + rg_pos(k / R)];
    const float2 zc = A[j * WS + (kc % R) * kRgRow + rg_pos(kc / R)];
    float re, im;
    if ((f & 1) == 0) {   // (Z[k] + conj Z[N-k]) / 2
      re = 0.5f * (zk.x + zc.x);
      im = 0.5f * (zk.y - zc.y);
    } else {              // (Z[k] - conj Z[N-k]) / (2i)
      re = 0.5f * (zk.y + zc.y);
      im = -0.5f * (zk.x - zc.x);
    }
    im += 0.f;   // -0 -> +0 (atan2 branch cut)
    const int o = k * T + t;
#if SE_RG_PROBE == 2   // probe: no spectrum stores (kept live by an impossible condition)
    if (re != 1234.5f) continue;
#endif
    if (!mag_phase) {
      if constexpr (!LP) {
        float* op = static_cast<float*>(out0) + ub;
#if SE_RG_NT
        __builtin_nontemporal_store(re, op + o);
        __builtin_nontemporal_store(im, op + o + half * T);
#else
        op[o] = re;
        op[o + half * T] = im;
#endif
      } else {
        stx<LP>(out0, ub + o, re, dt);
        stx<LP>(out0, ub + o + half * T, im, dt);
      }
    } else {
      stx<LP>(out0, ub + o, sqrtf(re * re + im * im), dt);
      stx<LP>(out1, ub + o, atan2f(im, re), dt);
    }
  }
}

// grid (ceil(T / 2 W PPW), B), 64 W threads. HALF: win <= N / 2 (registers q >= R/2 are zeros).
// PPW frame pairs per wave: their 64-point row passes run together, 8 R PPW butterflies over the
// wave's 64 lanes (R = 10, PPW = 2: 160 = 2.5 lane rounds per pass instead of 2 x 1.25)
template <int N, bool HALF, int W = 4, int PPW = 2, bool LP = false>
__global__ void __launch_bounds__(kWave * W) stft_fwd_rg_kernel(const StftArgs a) {
  constexpr int R = N / kWave, QN = HALF ? R / 2 : R, FT = 2 * W * PPW;
  static_assert(R * kWave == N, "nfft = 64 R");
  __shared__ __attribute__((aligned(16))) float2 A[W * PPW * R * kRgRow];
  int tb, b;
  xcd_frame_block(tb, b);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int t0 = tb * FT;
  const long long xo = (long long)b * a.L;
  const int pl = rg_pos(lane);
  float2* Aw = A + w * PPW * R * kRgRow;
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int ta = t0 + 2 * (w * PPW + p), tbb = ta + 1;
    float2 v[kMaxRadix];
#pragma unroll
    for (int q = QN; q < kMaxRadix; ++q) v[q] = make_float2(0.f, 0.f);
    const int sa = ta * a.hop - a.pad;
#if SE_RG_PROBE == 3   // probe: no signal loads
    if (true) {
#pragma unroll
      for (int q = 0; q < QN; ++q) v[q] = make_float2((float)(lane + q + tb), (float)(lane - q + b));
    } else
#endif
    if (!LP && sa >= 0 && tbb < a.T && sa + a.hop + a.win <= a.L) {
      const float* xp = static_cast<const float*>(a.x) + xo + sa;
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const int n = lane + q * kWave;
        const bool ok = n < a.win;
        const int nn = ok ? n : 0;
        const float wv = ok ? a.window[nn] : 0.f;
        v[q] = make_float2(wv * xp[nn], wv * xp[a.hop + nn]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const int n = lane + q * kWave;
        const bool ok = n < a.win;
        const int nn = ok ? n : 0;
        const float wv = ok ? a.window[nn] : 0.f;
        const float xa = ldx<LP>(a.x, xo + reflect_index(min(ta, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
        const float xb = ldx<LP>(a.x, xo + reflect_index(min(tbb, a.T - 1) * a.hop + nn - a.pad, a.L), a.dt);
        v[q] = make_float2(ta < a.T ? wv * xa : 0.f, tbb < a.T ? wv * xb : 0.f);
      }
    }
    float2 o[kMaxRadix];
    rdft<R>(v, o);
    float2* Ap = Aw + p * R * kRgRow;
    Ap[pl] = o[0];
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) Ap[k1 * kRgRow + pl] = cmul(o[k1], a.tw[lane * k1]);
  }
  wave_lds_sync();
#if SE_RG_PROBE != 1   // probe 1: no 64-point row passes
  rg_row_pass<R, 0, R * PPW>(Aw, a.tw, lane);
  rg_row_pass<R, 1, R * PPW>(Aw, a.tw, lane);
#endif
  __syncthreads();   // every pair of the block transformed
  rg_unpack_store<N, R, W * PPW, kWave * W, LP>(A, t0, a.T, b, a.out0, a.out1, a.mag_phase, a.dt);
}

struct IstftArgs {
  const void* in;      // fwd: spec [B, N+2, T]; bwd: gout [B, out_len]
  void* out;           // fwd: out [B, out_len]; bwd: gspec [B, N+2, T]
  int dt;              // SE_DTYPE_* of in / out
  const float* window;
  const float2* tw;
  int T, win, hop, offset, out_len, P, FT;
  FftPlan pl;
};

// Sums of v[f][n] over even / odd n < win for every frame f (one wave per frame).
// ysign scales the odd frames (the .y lanes), so a conjugate needs no separate pass.
__device__ void parity_sums(const float2* V, int P, int N, int win, float* sums /*[2P][2]*/,
                            float ysign = 1.f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int f = wave; f < 2 * P; f += nw) {
    const float2* v = V + (f >> 1) * N;
    float se = 0.f, so = 0.f;
    for (int n = lane; n < win; n += 64) {
      const float val = (f & 1) ? ysign * v[n].y : v[n].x;
      if (n & 1) so += val; else se += val;
    }
    se = se::wave_sum(se);
    so = se::wave_sum(so);
    if (lane == 0) { sums[2 * f] = se; sums[2 * f + 1] = so; }
  }
  __syncthreads();
}

// G = (M^T M)^{-1} applied to a frame: (v - e*Se/(a+ne) - o*So/(a+no)) / a
__device__ __forceinline__ float apply_g(float v, int n, float se_, float so_, float inv_a,
                                         float ce, float co) {
  return (v - ((n & 1) ? so_ * co : se_ * ce)) * inv_a;
}

// ConviSTFT forward. grid (ceil(out_len / (FT*hop)), B)
template <int CN, int CP, bool LP = false>
__global__ void __launch_bounds__(kThreads) istft_fwd_kernel(const IstftArgs a) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  __shared__ float sums[64];
  const int N = CN ? CN : a.pl.N, P = CP ? CP : a.P, half = N / 2 + 1;
  float2* A = lds;
  float2* Bf = lds + P * N;
  int sb, b;
  xcd_frame_block(sb, b);   // neighbouring sample tiles read the two halves of a row line
  const int s0 = a.offset + sb * a.FT * a.hop;
  const int s1 = min(s0 + a.FT * a.hop, a.offset + a.out_len);
  const int t_lo = max(0, ceil_div_i(s0 - a.win + 1, a.hop));
  const int t_hi = min(a.T - 1, floor_div(s1 - 1, a.hop));
  const long long so = (long long)b * 2 * half * a.T;

  // conj(C[k]) with C = E_a + i E_b, E the Hermitian completion of X / 2
  for (int idx = threadIdx.x; idx < half * P; idx += blockDim.x) {
    const int k = idx / P, j = idx - k * P;
    const int ta = t_lo + 2 * j, tb = ta + 1;
    float2 xa = make_float2(0.f, 0.f), xb = xa;
    if (ta <= t_hi) xa = make_float2(ldx<LP>(a.in, so + (long long)k * a.T + ta, a.dt),
                                     ldx<LP>(a.in, so + (long long)(half + k) * a.T + ta, a.dt));
    if (tb <= t_hi) xb = make_float2(ldx<LP>(a.in, so + (long long)k * a.T + tb, a.dt),
                                     ldx<LP>(a.in, so + (long long)(half + k) * a.T + tb, a.dt));
    float2* c = A + j * N;
    if (k == 0 || k == N / 2) {
      // E[k] = Re X[k]; C = Re Xa + i Re Xb; store conj
      c[k] = make_float2(xa.x, -xb.x);
    } else {
      // C[k] = Xa/2 + i Xb/2 ; C[N-k] = conj(Xa)/2 + i conj(Xb)/2
      const float2 ck = make_float2(0.5f * (xa.x - xb.y), 0.5f * (xa.y + xb.x));
      const float2 cn = make_float2(0.5f * (xa.x + xb.y), 0.5f * (-xa.y + xb.x));
      c[k] = make_float2(ck.x, -ck.y);
      c[N - k] = make_float2(cn.x, -cn.y);
    }
  }
  __syncthreads();
  float2* R = fft_any<CN, CP>(A, Bf, P, a.pl, a.tw);
  // z = conj(R): z_a = R.x, z_b = -R.y; the sign is folded into the sums and the frames.
  parity_sums(R, P, N, a.win, sums, -1.f);
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
  float* fr = reinterpret_cast<float*>(R == A ? Bf : A);   // [2P][win] frames
  for (int idx = threadIdx.x; idx < 2 * P * a.win; idx += blockDim.x) {
    const int f = idx / a.win, n = idx - f * a.win;
    const float2 z = R[(f >> 1) * N + n];
    const float v = (f & 1) ? -z.y : z.x;
    fr[idx] = a.window[n] * apply_g(v, n, sums[2 * f], sums[2 * f + 1], inv_a, ce, co);
  }
  __syncthreads();
  const long long oo = (long long)b * a.out_len;
  for (int s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
    const int tb0 = max(t_lo, ceil_div_i(s - a.win + 1, a.hop));
    const int tb1 = min(t_hi, floor_div(s, a.hop));
    float acc = 0.f, cf = 0.f;
    for (int t = tb0; t <= tb1; ++t) {
      const int n = s - t * a.hop;
      const float w = a.window[n];
      acc += fr[(t - t_lo) * a.win + n];
      cf += w * w;
    }
    stx<LP>(a.out, oo + s - a.offset, acc / (cf + 1e-8f), a.dt);
  }
}

// ConviSTFT forward on the in-place FFT (compiled plans): one P*N float2 LDS
// buffer holds the packed spectra, their FFT and then the windowed synthesis
// frames (written over it through registers), so a block needs ~half the LDS of
// istft_fwd_kernel and twice as many blocks share a CU. grid (ceil(out_len / (FT*hop)), B)
template <int CN, int P, bool LP = false>
__global__ void __launch_bounds__(kThreads) istft_fwd_ip_kernel(const IstftArgs a) {
  constexpr int N = CN, half = N / 2 + 1;
  __shared__ __attribute__((aligned(16))) float2 A[P * N];
  __shared__ float2 stw[N];
  __shared__ float sums[4 * P];
  int sb, b;
  xcd_frame_block(sb, b);
  const int s0 = a.offset + sb * a.FT * a.hop;
  const int s1 = min(s0 + a.FT * a.hop, a.offset + a.out_len);
  const int t_lo = max(0, ceil_div_i(s0 - a.win + 1, a.hop));
  const int t_hi = min(a.T - 1, floor_div(s1 - 1, a.hop));
  const long long so = (long long)b * 2 * half * a.T;
  for (int i = threadIdx.x; i < N; i += kThreads) stw[i] = a.tw[i];
  // spectrum gather: all of a thread's loads are issued before any is used
  // (compile-time trip count, clamped addresses, zeroed after the load)
  constexpr int GT = (half * P + kThreads - 1) / kThreads;
  float2 ga[GT], gb[GT];
#pragma unroll
  for (int it = 0; it < GT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    const int k = min(idx / P, half - 1), j = idx % P;
    const int ta = min(t_lo + 2 * j, t_hi), tb = min(t_lo + 2 * j + 1, t_hi);
    const long long re = so + (long long)k * a.T, im = so + (long long)(half + k) * a.T;
    ga[it] = make_float2(ldx<LP>(a.in, re + ta, a.dt), ldx<LP>(a.in, im + ta, a.dt));
    gb[it] = make_float2(ldx<LP>(a.in, re + tb, a.dt), ldx<LP>(a.in, im + tb, a.dt));
  }
  // conj(C[k]) with C = E_a + i E_b, E the Hermitian completion of X / 2
#pragma unroll
  for (int it = 0; it < GT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    if (idx >= half * P) break;
    const int k = idx / P, j = idx - k * P;
    const int ta = t_lo + 2 * j, tb = ta + 1;
    const float2 zero = make_float2(0.f, 0.f);
    const float2 xa = ta <= t_hi ? ga[it] : zero, xb = tb <= t_hi ? gb[it] : zero;
    float2* c = A + j * N;
    if (k == 0 || k == N / 2) {
      c[k] = make_float2(xa.x, -xb.x);
    } else {
      c[k] = make_float2(0.5f * (xa.x - xb.y), -0.5f * (xa.y + xb.x));
      c[N - k] = make_float2(0.5f * (xa.x + xb.y), 0.5f * (xa.y - xb.x));
    }
  }
  __syncthreads();
  fft_pass_ip<N, P, 0, 1>(A, stw);
  // z = conj(A): z_a = A.x, z_b = -A.y
  parity_sums(A, P, N, a.win, sums, -1.f);
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
  // frames fr[f][n] (n < win) over the same buffer: read all, barrier, write all
  constexpr int IT = (2 * P * N + kThreads - 1) / kThreads;
  float v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    const int f = idx / N, n = idx - f * N;
    v[it] = 0.f;
    if (idx < 2 * P * N && n < a.win) {
      const float2 z = A[(f >> 1) * N + n];
      v[it] = a.window[n] * apply_g((f & 1) ? -z.y : z.x, n, sums[2 * f], sums[2 * f + 1], inv_a, ce, co);
    }
  }
  __syncthreads();
  float* fr = reinterpret_cast<float*>(A);   // [2P][win]
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    const int f = idx / N, n = idx - f * N;
    if (idx < 2 * P * N && n < a.win) fr[f * a.win + n] = v[it];
  }
  __syncthreads();
  const long long oo = (long long)b * a.out_len;
  for (int s = s0 + threadIdx.x; s < s1; s += kThreads) {
    const int tb0 = max(t_lo, ceil_div_i(s - a.win + 1, a.hop));
    const int tb1 = min(t_hi, floor_div(s, a.hop));
    float acc = 0.f, cf = 0.f;
    for (int t = tb0; t <= tb1; ++t) {
      const int n = s - t * a.hop;
      const float w = a.window[n];
      acc += fr[(t - t_lo) * a.win + n];
      cf += w * w;
    }
    stx<LP>(a.out, oo + s - a.offset, acc / (cf + 1e-8f), a.dt);
  }
}

// Adjoint of istft_fwd. grid (ceil(T / 2P), B)
template <int CN, int CP, bool LP = false>
__global__ void __launch_bounds__(kThreads) istft_bwd_kernel(const IstftArgs a) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  __shared__ float sums[64];
  const int N = CN ? CN : a.pl.N, P = CP ? CP : a.P;
  float2* A = lds;
  float2* Bf = lds + P * N;
  int tb, b;
  xcd_frame_block(tb, b);
  const int t0 = tb * 2 * P;
  const long long go = (long long)b * a.out_len;
  for (int idx = threadIdx.x; idx < P * N; idx += blockDim.x) {
    const int j = idx / N, n = idx - j * N;
    float va = 0.f, vb = 0.f;
    if (n < a.win) {
      const float w = a.window[n];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = t0 + 2 * j + h;
        if (t >= a.T) continue;
        const int u = t * a.hop + n;
        if (u < a.offset || u >= a.offset + a.out_len) continue;
        // OLA normaliser at u (window^2 summed over covering frames)
        const int tb0 = max(0, ceil_div_i(u - a.win + 1, a.hop));
        const int tb1 = min(a.T - 1, floor_div(u, a.hop));
        float cf = 0.f;
        for (int tt = tb0; tt <= tb1; ++tt) {
          const float ww = a.window[u - tt * a.hop];
          cf += ww * ww;
        }
        const float v = w * ldx<LP>(a.in, go + u - a.offset, a.dt) / (cf + 1e-8f);
        if (h == 0) va = v; else vb = v;
      }
    }
    A[idx] = make_float2(va, vb);
  }
  __syncthreads();
  parity_sums(A, P, N, a.win, sums);
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
  for (int idx = threadIdx.x; idx < P * N; idx += blockDim.x) {
    const int j = idx / N, n = idx - j * N;
    if (n < a.win) {
      const float2 v = A[idx];
      A[idx] = make_float2(apply_g(v.x, n, sums[4 * j], sums[4 * j + 1], inv_a, ce, co),
                           apply_g(v.y, n, sums[4 * j + 2], sums[4 * j + 3], inv_a, ce, co));
    }
  }
  __syncthreads();
  const float2* Z = fft_any<CN, CP>(A, Bf, P, a.pl, a.tw);
  unpack_store<CN, CP, LP>(Z, P, N, t0, a.T, b, a.out, nullptr, 0, a.dt);
}

// istft_bwd on the in-place FFT (compiled plans): one P*N float2 LDS buffer,
// static LDS, twice the resident blocks of the ping-pong form. grid (ceil(T / 2P), B)
template <int CN, int P, bool LP = false>
__global__ void __launch_bounds__(kThreads) istft_bwd_ip_kernel(const IstftArgs a) {
  constexpr int N = CN;
  __shared__ __attribute__((aligned(16))) float2 A[P * N];
  __shared__ float2 stw[N];
  __shared__ float swin[N];
  __shared__ float sums[4 * P];
  int tb, b;
  xcd_frame_block(tb, b);
  const int t0 = tb * 2 * P;
  const long long go = (long long)b * a.out_len;
  for (int i = threadIdx.x; i < N; i += kThreads) {
    stw[i] = a.tw[i];
    swin[i] = i < a.win ? a.window[i] : 0.f;
  }
  // gradient gather: all of a thread's loads are issued first (compile-time trip
  // count, clamped addresses, masked after the load); the window is read from LDS
  constexpr int IT = (P * N + kThreads - 1) / kThreads;
  float ga[IT][2];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    const int j = idx / N, n = idx - j * N;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = (t0 + 2 * j + h) * a.hop + n;
      ga[it][h] = a.out_len > 0 ? ldx<LP>(a.in, go + min(max(u - a.offset, 0), a.out_len - 1), a.dt) : 0.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * kThreads;
    if (P * N % kThreads != 0 && idx >= P * N) break;
    const int j = idx / N, n = idx - j * N;
    float va = 0.f, vb = 0.f;
    if (n < a.win) {
      const float w = swin[n];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = t0 + 2 * j + h;
        if (t >= a.T) continue;
        const int u = t * a.hop + n;
        if (u < a.offset || u >= a.offset + a.out_len) continue;
        // OLA normaliser at u (window^2 summed over covering frames)
        const int tb0 = max(0, ceil_div_i(u - a.win + 1, a.hop));
        const int tb1 = min(a.T - 1, floor_div(u, a.hop));
        float cf = 0.f;
        for (int tt = tb0; tt <= tb1; ++tt) {
          const float ww = swin[u - tt * a.hop];
          cf += ww * ww;
        }
        const float v = w * ga[it][h] / (cf + 1e-8f);
        if (h == 0) va = v; else vb = v;
      }
    }
    A[idx] = make_float2(va, vb);
  }
  __syncthreads();
  parity_sums(A, P, N, a.win, sums);
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
  for (int idx = threadIdx.x; idx < P * N; idx += kThreads) {
    const int j = idx / N, n = idx - j * N;
    if (n < a.win) {
      const float2 v = A[idx];
      A[idx] = make_float2(apply_g(v.x, n, sums[4 * j], sums[4 * j + 1], inv_a, ce, co),
                           apply_g(v.y, n, sums[4 * j + 2], sums[4 * j + 3], inv_a, ce, co));
    }
  }
  __syncthreads();
  fft_pass_ip<N, P, 0, 1>(A, stw);
  unpack_store<N, P, LP>(A, P, N, t0, a.T, b, a.out, nullptr, 0, a.dt);
}

// ConviSTFT forward, wave-local FFT: W frame pairs per block. The spectrum gather
// (lanes along frames: coalesced row segments) and the overlap-add store are
// block-wide; each wave transforms its pair, takes its frames' parity sums and
// writes its two synthesis frames without a block barrier.
// grid (ceil(out_len / (FT*hop)), B), FT = 2W - 1 - (win-1)/hop, 64 W threads
// RG: the pair's FFT is the register-radix one of stft_fwd_rg_kernel (nfft = 64 R): lane l
// takes C[l + 64 q] of its pair into registers, and the frame comes back in the row image
// (sample n at row n % R, column n / R); pair stride R x kRgRow.
template <int CN, int W = wv_pairs<CN>(), bool LP = false, bool RG = false>
__global__ void __launch_bounds__(kWave * W) istft_fwd_wv_kernel(const IstftArgs a) {
  constexpr int N = CN, TPB = kWave * W, half = N / 2 + 1, P = W;
  constexpr int R = RG ? N / kWave : 1, NP = RG ? R * kRgRow : wv_stride<N>();
  static_assert(!RG || R * kWave == N, "nfft = 64 R");
  __shared__ __attribute__((aligned(16))) float2 A[W * NP];
#if SE_STFT_TWL_IFWD
  __shared__ float2 stw[N];
#else
  const float2* stw = a.tw;
#endif
  int sb, b;
  xcd_frame_block(sb, b);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int s0 = a.offset + sb * a.FT * a.hop;
  const int s1 = min(s0 + a.FT * a.hop, a.offset + a.out_len);
  const int t_lo = max(0, ceil_div_i(s0 - a.win + 1, a.hop));
  const int t_hi = min(a.T - 1, floor_div(s1 - 1, a.hop));
  const long long so = (long long)b * 2 * half * a.T;
  // spectrum gather, all loads issued first (clamped addresses, zeroed after the load)
  constexpr int GT = (half * P + TPB - 1) / TPB;
  float2 ga[GT], gb[GT];
#pragma unroll
  for (int it = 0; it < GT; ++it) {
    const int idx = threadIdx.x + it * TPB;
    const int k = min(idx / P, half - 1), j = idx % P;
    const int ta = min(t_lo + 2 * j, t_hi), tb = min(t_lo + 2 * j + 1, t_hi);
    const int re = k * a.T, im = (half + k) * a.T;   // 32-bit offsets within the utterance
    if constexpr (!LP) {
      const float* sp = static_cast<const float*>(a.in) + so;
      ga[it] = make_float2(sp[re + ta], sp[im + ta]);
      gb[it] = make_float2(sp[re + tb], sp[im + tb]);
    } else {
      ga[it] = make_float2(ldx<LP>(a.in, so + re + ta, a.dt), ldx<LP>(a.in, so + im + ta, a.dt));
      gb[it] = make_float2(ldx<LP>(a.in, so + re + tb, a.dt), ldx<LP>(a.in, so + im + tb, a.dt));
    }
  }
#if SE_STFT_TWL_IFWD
  for (int i = threadIdx.x; i < N; i += TPB) stw[i] = a.tw[i];
#endif
  // conj(C[k]) with C = E_a + i E_b, E the Hermitian completion of X / 2
#pragma unroll
  for (int it = 0; it < GT; ++it) {
    const int idx = threadIdx.x + it * TPB;
    if (idx >= half * P) break;
    const int k = idx / P, j = idx - k * P;
    const int ta = t_lo + 2 * j, tb = ta + 1;
    const float2 zero = make_float2(0.f, 0.f);
    const float2 xa = ta <= t_hi ? ga[it] : zero, xb = tb <= t_hi ? gb[it] : zero;
    float2* c = A + j * NP;
    if (k == 0 || k == N / 2) {
      c[k] = make_float2(xa.x, -xb.x);
    } else {
      c[k] = make_float2(0.5f * (xa.x - xb.y), -0.5f * (xa.y + xb.x));
      c[N - k] = make_float2(0.5f * (xa.x + xb.y), 0.5f * (xa.y - xb.x));
    }
  }
  __syncthreads();
  float2* Aw = A + w * NP;
  if constexpr (RG) {
    float2 v[kMaxRadix], o[kMaxRadix];
#pragma unroll
    for (int q = 0; q < kMaxRadix; ++q) v[q] = q < R ? Aw[lane + q * kWave] : make_float2(0.f, 0.f);
    wave_lds_sync();   // the whole pair read before the row image overwrites it
    rdft<R>(v, o);
    const int pl = rg_pos(lane);
    Aw[pl] = o[0];
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) Aw[k1 * kRgRow + pl] = cmul(o[k1], a.tw[lane * k1]);
    wave_lds_sync();
    rg_row_pass<R, 0, R>(Aw, a.tw, lane);
    rg_row_pass<R, 1, R>(Aw, a.tw, lane);
  } else {
    wfft_pass<N, 0, 1>(Aw, stw, lane);
  }
  // z = conj(Aw): z_a = Aw.x, z_b = -Aw.y. Parity sums over n < win, then the
  // windowed G-corrected frames written over the wave's own buffer as [2][win] floats
  constexpr int IT = (N + kWave - 1) / kWave;
  float2 z[IT];
  float sea = 0.f, soa = 0.f, seb = 0.f, sob = 0.f;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    // RG: lane l takes samples n = R l + it (row it, column l of the image: conflict-free)
    const int n = RG ? lane * R + it : lane + it * kWave;
    z[it] = n < a.win ? Aw[RG ? it * kRgRow + rg_pos(lane) : n] : make_float2(0.f, 0.f);
    z[it].y = -z[it].y;
    if (n & 1) { soa += z[it].x; sob += z[it].y; } else { sea += z[it].x; seb += z[it].y; }
  }
  sea = se::wave_sum(sea); soa = se::wave_sum(soa);
  seb = se::wave_sum(seb); sob = se::wave_sum(sob);
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
  wave_lds_sync();
  float* fw = reinterpret_cast<float*>(Aw);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int n = RG ? lane * R + it : lane + it * kWave;
    if (n < a.win) {
      const float wn = a.window[n];
      fw[n] = wn * apply_g(z[it].x, n, sea, soa, inv_a, ce, co);
      fw[a.win + n] = wn * apply_g(z[it].y, n, seb, sob, inv_a, ce, co);
    }
  }
  __syncthreads();
  const long long oo = (long long)b * a.out_len;
  const float rh = 1.f / (float)a.hop;
  for (int s = s0 + threadIdx.x; s < s1; s += TPB) {
    // covering frames [tb0, tb1] of sample s: s = q hop + r; frame t covers it while
    // s - t hop < win, i.e. t >= q - floor((win - 1 - r) / hop) (none if r >= win)
    const int q = fdiv_nn(s, a.hop, rh), m = a.win - 1 - (s - q * a.hop);
    const int tb0 = max(t_lo, m < 0 ? q + 1 : q - fdiv_nn(m, a.hop, rh));
    const int tb1 = min(t_hi, q);
    float acc = 0.f, cf = 0.f;
    for (int t = tb0; t <= tb1; ++t) {
      const int n = s - t * a.hop, f = t - t_lo;
      const float wn = a.window[n];
      acc += reinterpret_cast<const float*>(A + (f >> 1) * NP)[(f & 1) * a.win + n];
      cf += wn * wn;
    }
    stx<LP>(a.out, oo + s - a.offset, acc / (cf + 1e-8f), a.dt);
  }
}

// The adjoint's frame side, shared by istft_bwd_wv_kernel and istft_bwd_rg_kernel: wave w
// gathers frames t0 + 2w, +1 from the output gradient (contiguous samples: coalesced),
// divides by the OLA normaliser, windows and applies G with the frames' own parity sums.
// g[it][h] = sample n = lane + 64 it of frame h (zero for n >= win); iterations it >= QI are
// not formed (the caller knows them zero: win <= 64 QI). Stages the window in swin (one
// block barrier, before which the caller may stage more).
template <int N, int QI, bool LP>
__device__ __forceinline__ void ibwd_frames(const IstftArgs& a, float* swin, int b, int t0, int w, int lane,
                                            float (&g)[QI][2]) {
  const long long go = (long long)b * a.out_len;
  float ga[QI][2];
#pragma unroll
  for (int it = 0; it < QI; ++it) {
    const int n = lane + it * kWave;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ga[it][h] = 0.f;
      if (it * kWave < a.win && a.out_len > 0) {   // wave-uniform: frame samples n < win only
        const int u = (t0 + 2 * w + h) * a.hop + min(n, a.win - 1);
        ga[it][h] = ldx<LP>(a.in, go + min(max(u - a.offset, 0), a.out_len - 1), a.dt);
      }
    }
  }
  for (int i = threadIdx.x; i < N; i += blockDim.x) swin[i] = i < a.win ? a.window[i] : 0.f;
  __syncthreads();
  float v[QI][2];
  float se2[2] = {0.f, 0.f}, so2[2] = {0.f, 0.f};
  const float rh = 1.f / (float)a.hop;
#pragma unroll
  for (int it = 0; it < QI; ++it) {
    const int n = lane + it * kWave;
    // frames t + d covering sample u = t hop + n: d in [d0, d1] (n < win), the same
    // for both of the wave's frames up to the clip to [0, T - 1]
    const int nc = min(n, a.win - 1);
    const int d1 = fdiv_nn(nc, a.hop, rh), d0 = -fdiv_nn(a.win - 1 - nc, a.hop, rh);
    // OLA normaliser at u (window^2 summed over the covering frames, in frame order): the
    // same for both frames unless a frame sits at a signal end (clipped range)
    float cfi = 0.f;
    for (int d = d0; d <= d1; ++d) {
      const float ww = swin[n - d * a.hop];
      cfi += ww * ww;
    }
    const float wn = swin[nc];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float val = 0.f;
      const int t = t0 + 2 * w + h;
      const int u = t * a.hop + n;
      if (n < a.win && t < a.T && u >= a.offset && u < a.offset + a.out_len) {
        float cf = cfi;
        if (t + d0 < 0 || t + d1 > a.T - 1) {
          cf = 0.f;
          for (int d = max(d0, -t); d <= min(d1, a.T - 1 - t); ++d) {
            const float ww = swin[n - d * a.hop];
            cf += ww * ww;
          }
        }
        val = wn * ga[it][h] / (cf + 1e-8f);
      }
      v[it][h] = val;
      if (n & 1) so2[h] += val; else se2[h] += val;
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) { se2[h] = se::wave_sum(se2[h]); so2[h] = se::wave_sum(so2[h]); }
  const float ah = 0.5f * N, inv_a = 1.f / ah;
  const float ce = 1.f / (ah + (a.win + 1) / 2), co = 1.f / (ah + a.win / 2);
#pragma unroll
  for (int it = 0; it < QI; ++it) {
    const int n = lane + it * kWave;
    const bool in = n < a.win;
#pragma unroll
    for (int h = 0; h < 2; ++h) g[it][h] = in ? apply_g(v[it][h], n, se2[h], so2[h], inv_a, ce, co) : 0.f;
  }
}

// Adjoint of istft_fwd, wave-local FFT: wave w forms its frame pair (ibwd_frames) and
// transforms it; one barrier before the block-wide spectrum store.
// grid (ceil(T / 2W), B), 64 W threads
template <int CN, int W = wv_pairs<CN>(), bool LP = false>
__global__ void __launch_bounds__(kWave * W) istft_bwd_wv_kernel(const IstftArgs a) {
  constexpr int N = CN, NP = wv_stride<N>();
  __shared__ __attribute__((aligned(16))) float2 A[W * NP];
#if SE_STFT_TWL_IBWD
  __shared__ float2 stw[N];
  for (int i = threadIdx.x; i < N; i += kWave * W) stw[i] = a.tw[i];
#else
  const float2* stw = a.tw;
#endif
  __shared__ float swin[N];
  int tb, b;
  xcd_frame_block(tb, b);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int t0 = tb * 2 * W;
  constexpr int IT = (N + kWave - 1) / kWave;
  float g[IT][2];
  ibwd_frames<N, IT, LP>(a, swin, b, t0, w, lane, g);
  float2* Aw = A + w * NP;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int n = lane + it * kWave;
    if (N % kWave == 0 || n < N) Aw[n] = make_float2(g[it][0], g[it][1]);
  }
  wave_lds_sync();
  wfft_pass<N, 0, 1>(Aw, stw, lane);
  __syncthreads();
  wv_unpack_store<N, W, LP>(A, t0, a.T, b, a.out, nullptr, 0, a.dt);
}

// Adjoint of istft_fwd with the register-radix FFT of stft_fwd_rg_kernel (nfft = 64 R):
// ibwd_frames leaves lane l samples l + 64 q of its wave's two frames in registers, which is
// the register-radix input layout, so the R-point DFT runs straight on them (no LDS image
// before the first stage, and with HALF (win <= N / 2) the upper R / 2 inputs are compile-time
// zeros); then the two 64-point row passes and the shared unpack store.
// grid (ceil(T / 2W), B), 64 W threads
template <int N, bool HALF, int W, bool LP>
__global__ void __launch_bounds__(kWave * W) istft_bwd_rg_kernel(const IstftArgs a) {
  constexpr int R = N / kWave, QN = HALF ? R / 2 : R;
  static_assert(R * kWave == N, "nfft = 64 R");
  __shared__ __attribute__((aligned(16))) float2 A[W * R * kRgRow];
  __shared__ float swin[N];
  int tb, b;
  xcd_frame_block(tb, b);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int t0 = tb * 2 * W;
  float g[QN][2];
  ibwd_frames<N, QN, LP>(a, swin, b, t0, w, lane, g);
  float2 v[kMaxRadix], o[kMaxRadix];
#pragma unroll
  for (int q = 0; q < kMaxRadix; ++q) v[q] = q < QN ? make_float2(g[q][0], g[q][1]) : make_float2(0.f, 0.f);
  rdft<R>(v, o);
  float2* Aw = A + w * R * kRgRow;
  const int pl = rg_pos(lane);
  Aw[pl] = o[0];
#pragma unroll
  for (int k1 = 1; k1 < R; ++k1) Aw[k1 * kRgRow + pl] = cmul(o[k1], a.tw[lane * k1]);
  wave_lds_sync();
  rg_row_pass<R, 0, R>(Aw, a.tw, lane);
  rg_row_pass<R, 1, R>(Aw, a.tw, lane);
  __syncthreads();   // every pair of the block transformed
  rg_unpack_store<N, R, W, kWave * W, LP>(A, t0, a.T, b, a.out, nullptr, 0, a.dt);
}

// ---------------------------------------------------------------------------
static bool make_plan(int N, FftPlan& pl) {
  if (N < 2 || N > 1024) return false;
  pl.N = N;
  pl.npass = 0;
  int n = N;
  const int order[4] = {4, 2, 3, 5};
  for (int r : order) {
    while (n % r == 0) {
      if (pl.npass >= kMaxPasses) return false;
      pl.radix[pl.npass++] = r;
      n /= r;
    }
  }
  return n == 1;
}

// Frame pairs per block. kPairs (4) keeps a block's LDS at <= 40 KB for
// nfft <= 640 so four blocks (16 waves) share a CU; larger nfft fall back to
// what the LDS budget allows.
constexpr int kPairs = 4;
// the compiled radix plans run the in-place kernels
static bool ip_plan(int nfft) { return nfft == 640 || nfft == 512 || nfft == 400 || nfft == 320 || nfft == 256; }
static int pick_pairs(int N) {
  const int p = kLdsBudget / (2 * N * (int)sizeof(float2));
  return std::max(1, std::min(kPairs, p));   // sums[] holds 2 floats for 32 frames
}

// Launch K<CN, CP, LP> for the compiled plans (CP = kPairs), else K<0, 0, LP>;
// LP = the tensors are bf16 / fp16 (a.dt != SE_DTYPE_F32).
#define SE_COMMA ,
#define SE_LP_LAUNCH(K, grid, shm, st, a)                                                           \
  do {                                                                                             \
    if ((a).dt != SE_DTYPE_F32) hipLaunchKernelGGL((K, true>), grid, dim3(kThreads), shm, st, a);  \
    else hipLaunchKernelGGL((K, false>), grid, dim3(kThreads), shm, st, a);                        \
  } while (0)
#define SE_STFT_DISPATCH(K, nfft, P, grid, shm, st, a)                                              \
  do {                                                                                             \
    const bool cp_ = (P) == kPairs;                                                                \
    switch (cp_ ? (nfft) : 0) {                                                                    \
      case 640: SE_LP_LAUNCH(K<640 SE_COMMA kPairs, grid, shm, st, a); break;                      \
      case 512: SE_LP_LAUNCH(K<512 SE_COMMA kPairs, grid, shm, st, a); break;                      \
      case 400: SE_LP_LAUNCH(K<400 SE_COMMA kPairs, grid, shm, st, a); break;                      \
      case 320: SE_LP_LAUNCH(K<320 SE_COMMA kPairs, grid, shm, st, a); break;                      \
      case 256: SE_LP_LAUNCH(K<256 SE_COMMA kPairs, grid, shm, st, a); break;                      \
      default: SE_LP_LAUNCH(K<0 SE_COMMA 0, grid, shm, st, a); break;                              \
    }                                                                                              \
  } while (0)
static int dtype_ok(int dt) { return dt == SE_DTYPE_F32 || dt == SE_DTYPE_BF16 || dt == SE_DTYPE_F16; }

static int check_common(int win, int hop, int nfft, FftPlan& pl) {
  if (win <= 0 || hop <= 0 || nfft <= 0 || win > nfft) return SE_E_ARG;
  if (nfft & 1) return SE_E_UNSUPPORTED;   // the pinv closed form assumes a Nyquist bin
  if (!make_plan(nfft, pl)) return SE_E_UNSUPPORTED;
  return SE_OK;
}

}  // namespace

extern "C" int se_stft_num_frames(int L, int win, int hop, int nfft, int center) {
  if (L <= 0 || win <= 0 || hop <= 0 || nfft <= 0) return -1;
  const int pad = center ? nfft / 2 : 0;
  const int Lp = L + 2 * pad;
  if (Lp < win) return 0;
  return (Lp - win) / hop + 1;
}

extern "C" int se_stft_fwd(const void* x, void* out0, void* out1, int B, int L, int win,
                           int hop, int nfft, int center, int mag_phase, const float* window,
                           const float* twiddle, int dtype, void* stream) {
  FftPlan pl;
  int rc = check_common(win, hop, nfft, pl);
  if (rc) return rc;
  if (!x || !out0 || !window || !twiddle || B <= 0 || L <= 0 || (mag_phase && !out1) || !dtype_ok(dtype))
    return SE_E_ARG;
  const int pad = center ? nfft / 2 : 0;
  if (center && L <= pad) return SE_E_SHAPE;   // reflect pad needs L > pad (F.pad reflect)
  const int T = se_stft_num_frames(L, win, hop, nfft, center);
  if (T <= 0) return SE_E_SHAPE;
  StftArgs a{};
  a.x = x; a.out0 = out0; a.out1 = out1; a.window = window; a.tw = (const float2*)twiddle; a.dt = dtype;
  a.L = L; a.win = win; a.hop = hop; a.T = T; a.pad = pad; a.mag_phase = mag_phase;
  a.P = pick_pairs(nfft); a.pl = pl;
  const size_t shm = 2 * (size_t)a.P * nfft * sizeof(float2);
  if (SE_STFT_RG && (nfft == 640 || nfft == 512 || nfft == 320)) {
    hipStream_t st = se::as_stream(stream);
    constexpr int W = SE_RG_W, PPW = SE_RG_PPW;
    const dim3 grid(se::ceil_div(T, 2 * W * PPW), B), blk(se::kWave * W);
    const bool hf = 2 * win <= nfft;
#define SE_STFT_RGL(NF, H)                                                                              \
    do {                                                                                                \
      if (a.dt != SE_DTYPE_F32) hipLaunchKernelGGL((stft_fwd_rg_kernel<NF, H, W, PPW, true>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((stft_fwd_rg_kernel<NF, H, W, PPW, false>), grid, blk, 0, st, a);         \
    } while (0)
    if (nfft == 640) { if (hf) SE_STFT_RGL(640, true); else SE_STFT_RGL(640, false); }
    else if (nfft == 512) { if (hf) SE_STFT_RGL(512, true); else SE_STFT_RGL(512, false); }
    else SE_STFT_RGL(320, false);
#undef SE_STFT_RGL
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  if (SE_STFT_WV && ip_plan(nfft)) {
    // wave-local FFT, wv_pairs<nfft>() frame pairs per block
    hipStream_t st = se::as_stream(stream);
#define SE_STFT_WVL(NF)                                                                                 \
    do {                                                                                                \
      constexpr int W = wv_pairs<NF>();                                                                 \
      const dim3 grid(se::ceil_div(T, 2 * W), B), blk(se::kWave * W);                                   \
      if (a.dt != SE_DTYPE_F32) hipLaunchKernelGGL((stft_fwd_wv_kernel<NF, W, true>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((stft_fwd_wv_kernel<NF, W, false>), grid, blk, 0, st, a);                 \
    } while (0)
    switch (nfft) {
      case 640: SE_STFT_WVL(640); break;
      case 512: SE_STFT_WVL(512); break;
      case 400: SE_STFT_WVL(400); break;
      case 320: SE_STFT_WVL(320); break;
      default: SE_STFT_WVL(256); break;
    }
#undef SE_STFT_WVL
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  if (ip_plan(nfft)) {
    // in-place FFT, kPairsIP frame pairs per block (static LDS <= 25 KB)
    const int P = kPairsIP;
    const dim3 grid(se::ceil_div(T, 2 * P), B);
    hipStream_t st = se::as_stream(stream);
#define SE_STFT_IP(NF) SE_LP_LAUNCH(stft_fwd_ip_kernel<NF SE_COMMA kPairsIP, grid, 0, st, a)
    switch (nfft) {
      case 640: SE_STFT_IP(640); break;
      case 512: SE_STFT_IP(512); break;
      case 400: SE_STFT_IP(400); break;
      case 320: SE_STFT_IP(320); break;
      default: SE_STFT_IP(256); break;
    }
#undef SE_STFT_IP
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  SE_STFT_DISPATCH(stft_fwd_kernel, nfft, a.P, dim3(se::ceil_div(T, 2 * a.P), B), shm, se::as_stream(stream), a);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

static int istft_setup(int B, int T, int win, int hop, int nfft, int offset, int out_len,
                       IstftArgs& a) {
  FftPlan pl;
  int rc = check_common(win, hop, nfft, pl);
  if (rc) return rc;
  if (B <= 0 || T <= 0 || offset < 0 || out_len < 0) return SE_E_ARG;
  if (offset + out_len > (T - 1) * hop + win) return SE_E_SHAPE;
  a.T = T; a.win = win; a.hop = hop; a.offset = offset; a.out_len = out_len;
  a.P = pick_pairs(nfft); a.pl = pl;
  // output tile of the generic forward kernel: the covering frames of FT*hop
  // samples must fit in 2P (checked where that kernel launches; the in-place
  // kernels use their own P, the adjoint tiles by frames)
  a.FT = 2 * a.P - 1 - (win - 1) / hop;
  return SE_OK;
}

extern "C" int se_istft_fwd(const void* spec, void* out, int B, int T, int win, int hop,
                            int nfft, int offset, int out_len, const float* window,
                            const float* twiddle, int dtype, void* stream) {
  IstftArgs a{};
  int rc = istft_setup(B, T, win, hop, nfft, offset, out_len, a);
  if (rc) return rc;
  if (!spec || !out || !window || !twiddle || !dtype_ok(dtype)) return SE_E_ARG;
  if (out_len == 0) return SE_OK;
  a.in = spec; a.out = out; a.window = window; a.tw = (const float2*)twiddle; a.dt = dtype;
  if (SE_STFT_WV && ip_plan(nfft)) {
    // wave-local FFT, wv_pairs<nfft>() frame pairs per block
    const int W = nfft == 640 ? wv_pairs<640>() : nfft == 512 ? wv_pairs<512>() : nfft == 400 ? wv_pairs<400>()
                : nfft == 320 ? wv_pairs<320>() : wv_pairs<256>();
    a.P = W;
    a.FT = 2 * W - 1 - (win - 1) / hop;
    if (a.FT >= 1) {
      const dim3 grid(se::ceil_div(out_len, a.FT * hop), B), blk(se::kWave * W);
      hipStream_t st = se::as_stream(stream);
#define SE_ISTFT_WVL(NF, G)                                                                             \
      do {                                                                                              \
        if (a.dt != SE_DTYPE_F32) hipLaunchKernelGGL((istft_fwd_wv_kernel<NF, wv_pairs<NF>(), true, G>), grid, blk, 0, st, a); \
        else hipLaunchKernelGGL((istft_fwd_wv_kernel<NF, wv_pairs<NF>(), false, G>), grid, blk, 0, st, a); \
      } while (0)
      switch (nfft) {
        case 640: SE_ISTFT_WVL(640, SE_ISTFT_FWD_RG); break;
        case 512: SE_ISTFT_WVL(512, SE_ISTFT_FWD_RG); break;
        case 400: SE_ISTFT_WVL(400, false); break;
        case 320: SE_ISTFT_WVL(320, SE_ISTFT_FWD_RG); break;
        default: SE_ISTFT_WVL(256, false); break;
      }
#undef SE_ISTFT_WVL
      SE_LAUNCH_CHECK();
      return SE_OK;
    }
  }
  if (ip_plan(nfft)) {
    // in-place FFT, kPairsIP frame pairs per block (8 measured slower: 79.9 / 107 us)
    const int P = kPairsIP;
    a.P = P;
    a.FT = 2 * P - 1 - (win - 1) / hop;
    if (a.FT >= 1) {
      const dim3 grid(se::ceil_div(out_len, a.FT * hop), B);
      hipStream_t st = se::as_stream(stream);
#define SE_ISTFT_IP(NF) SE_LP_LAUNCH(istft_fwd_ip_kernel<NF SE_COMMA kPairsIP, grid, 0, st, a)
      switch (nfft) {
        case 640: SE_ISTFT_IP(640); break;
        case 512: SE_ISTFT_IP(512); break;
        case 400: SE_ISTFT_IP(400); break;
        case 320: SE_ISTFT_IP(320); break;
        default: SE_ISTFT_IP(256); break;
      }
#undef SE_ISTFT_IP
      SE_LAUNCH_CHECK();
      return SE_OK;
    }
    istft_setup(B, T, win, hop, nfft, offset, out_len, a);   // FT too small at this P: generic kernel
  }
  if (a.FT < 1) return SE_E_UNSUPPORTED;
  const size_t shm = 2 * (size_t)a.P * nfft * sizeof(float2);
  SE_STFT_DISPATCH(istft_fwd_kernel, nfft, a.P, dim3(se::ceil_div(out_len, a.FT * hop), B), shm,
                   se::as_stream(stream), a);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_istft_bwd(const void* gout, void* gspec, int B, int T, int win, int hop,
                            int nfft, int offset, int out_len, const float* window,
                            const float* twiddle, int dtype, void* stream) {
  IstftArgs a{};
  int rc = istft_setup(B, T, win, hop, nfft, offset, out_len, a);
  if (rc) return rc;
  if (!gout || !gspec || !window || !twiddle || !dtype_ok(dtype)) return SE_E_ARG;
  a.in = gout; a.out = gspec; a.window = window; a.tw = (const float2*)twiddle; a.dt = dtype;
  if (SE_ISTFT_BWD_RG && (nfft == 640 || nfft == 512 || nfft == 320)) {
    // register-radix FFT, SE_IRG_W frame pairs per block
    hipStream_t st = se::as_stream(stream);
    constexpr int W = SE_IRG_W;
    const dim3 grid(se::ceil_div(T, 2 * W), B), blk(se::kWave * W);
    const bool hf = 2 * win <= nfft;
#define SE_ISTFT_RGL(NF, H)                                                                             \
    do {                                                                                                \
      if (a.dt != SE_DTYPE_F32) hipLaunchKernelGGL((istft_bwd_rg_kernel<NF, H, W, true>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((istft_bwd_rg_kernel<NF, H, W, false>), grid, blk, 0, st, a);             \
    } while (0)
    if (nfft == 640) { if (hf) SE_ISTFT_RGL(640, true); else SE_ISTFT_RGL(640, false); }
    else if (nfft == 512) { if (hf) SE_ISTFT_RGL(512, true); else SE_ISTFT_RGL(512, false); }
    else SE_ISTFT_RGL(320, false);
#undef SE_ISTFT_RGL
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  if (SE_STFT_WV && ip_plan(nfft)) {
    // wave-local FFT, wv_pairs<nfft>() frame pairs per block
    hipStream_t st = se::as_stream(stream);
#define SE_ISTFT_BWD_WVL(NF)                                                                            \
    do {                                                                                                \
      constexpr int W = wv_pairs<NF>();                                                                 \
      const dim3 grid(se::ceil_div(T, 2 * W), B), blk(se::kWave * W);                                   \
      if (a.dt != SE_DTYPE_F32) hipLaunchKernelGGL((istft_bwd_wv_kernel<NF, W, true>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((istft_bwd_wv_kernel<NF, W, false>), grid, blk, 0, st, a);               \
    } while (0)
    switch (nfft) {
      case 640: SE_ISTFT_BWD_WVL(640); break;
      case 512: SE_ISTFT_BWD_WVL(512); break;
      case 400: SE_ISTFT_BWD_WVL(400); break;
      case 320: SE_ISTFT_BWD_WVL(320); break;
      default: SE_ISTFT_BWD_WVL(256); break;
    }
#undef SE_ISTFT_BWD_WVL
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  if (ip_plan(nfft)) {
    // in-place FFT, kPairsIP frame pairs per block (8 measured slower: 79.9 / 107 us)
    const int P = kPairsIP;
    const dim3 grid(se::ceil_div(T, 2 * P), B);
    hipStream_t st = se::as_stream(stream);
#define SE_ISTFT_BWD_IP(NF) SE_LP_LAUNCH(istft_bwd_ip_kernel<NF SE_COMMA kPairsIP, grid, 0, st, a)
    switch (nfft) {
      case 640: SE_ISTFT_BWD_IP(640); break;
      case 512: SE_ISTFT_BWD_IP(512); break;
      case 400: SE_ISTFT_BWD_IP(400); break;
      case 320: SE_ISTFT_BWD_IP(320); break;
      default: SE_ISTFT_BWD_IP(256); break;
    }
#undef SE_ISTFT_BWD_IP
    SE_LAUNCH_CHECK();
    return SE_OK;
  }
  const size_t shm = 2 * (size_t)a.P * nfft * sizeof(float2);
  SE_STFT_DISPATCH(istft_bwd_kernel, nfft, a.P, dim3(se::ceil_div(T, 2 * a.P), B), shm, se::as_stream(stream), a);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
