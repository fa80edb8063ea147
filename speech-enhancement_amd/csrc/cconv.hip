// Complex (transposed) 2-D convolution as one fused implicit GEMM on MFMA.
//
// Replaces ComplexConv.forward (complex_nn.py:52-65) — four real
// nn.Conv2d / nn.ConvTranspose2d calls plus sub/add/cat — and their autograd
// backward, for ComplexConv2d (complex_nn.py:67-78) and
// ComplexConvTranspose2d (complex_nn.py:80-91); also plain real convs
// (frcrn.py:115 final_conv) when complex_weights == 0.
//
// Every pass (forward, data-grad) is an OUTPUT-STATIONARY GATHER GEMM
//   Y[b, n, p_h + S_h*q_h, p_w + S_w*q_w] = sum_k G[m, k] * Wp[k, n]
//   m = (b, q_h, q_w),  k = tap * Cg + c,
//   G[m, k] = X[b, c, q_h*s_h + off_h[tap], q_w*s_w + off_w[tap]]   (0 outside)
// A strided conv is one class (S = 1, s = stride). A transposed conv (and a
// conv's data-grad) is split into stride-phase classes p (S = stride, s = 1)
// whose tap lists keep only the kernel rows that hit that phase, so no MFMA
// work is spent on the zeros a naive "dilate then convolve" would insert.
// The weight-grad pass is a reduction GEMM over m:
//   dWp[k, n] = sum_m G[m, k] * D[m, n]
//
// Tiles: fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32 (exact fp32,
// no TF32 on gfx950). A workgroup of 4 waves computes BN x BM outputs; the
// MFMA A operand is the weight tile (rows = n), the B operand the gathered
// activations (cols = m) so the accumulator's lane index runs along m = the
// contiguous time axis and epilogue stores are 128-B coalesced.
#include "common.hpp"

#include <mutex>

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kThreads = 256;
constexpr int kBK = 32;      // reduction depth per K-step (16 MFMA k-pairs)
constexpr int kMaxTaps = 64; // per-class taps (kh*kw <= 64)
constexpr int kInvalidOff = -(1 << 29);

typedef float f32x4 __attribute__((ext_vector_type(4)));   // native vector (SROA-friendly)
typedef float f32x2 __attribute__((ext_vector_type(2)));
// Out-of-range gather lanes read a zeroed page of the workspace (global
// memory, like the tensors, so the select stays a global_load) instead of
// selecting after the load: the loaded register then feeds the LDS write
// directly and the load stays in flight across the MFMA loop.
constexpr size_t kZeroBytes = 256;
constexpr size_t kAmaxBytes = 256;   // SE_MATH_F16X3 max |.| slots, zeroed only when a pass fills one

// The zero page lives once per device (allocated and cleared on first use, never
// written), not in the workspace: a per-call hipMemsetAsync was a fill launch on
// the caller's stream before every conv pass, and in the backward each such
// launch waits for a CU slot beside the side-stream weight-grads.
static const float* zero_page() {
  static std::mutex mu;
  static void* pages[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!pages[dev]) {
    void* q = nullptr;
    if (hipMalloc(&q, kZeroBytes) != hipSuccess) return nullptr;
    if (hipMemset(q, 0, kZeroBytes) != hipSuccess) { (void)hipFree(q); return nullptr; }
    pages[dev] = q;
  }
  return (const float*)pages[dev];
}

// ---------------------------------------------------------------------------
// Gather-GEMM (forward and data-grad)
// ---------------------------------------------------------------------------
// XCD-aware workgroup order. Workgroups are dispatched round-robin over the 8
// XCDs, each with its own L2, so consecutive linear ids land on different L2s
// and neighbouring tiles (which share gathered input rows across taps, or the
// D rows of one weight-grad split) miss each other's lines. This bijection on
// [0, total) gives each XCD a contiguous range of logical tiles; it is a pure
// relabelling, so results do not depend on the actual dispatch order.
// Each GEMM K-step is one scheduling region whose non-MFMA instructions are
// interleaved into the MFMA gaps by sched_group_barrier groups (gather fwd/dgrad
// +6-9 %, weight-grad +6 % over a fenced schedule).
__device__ __forceinline__ int xcd_remap(int L, int total) {
  constexpr int kXcd = 8;
  const int xcd = L % kXcd, idx = L / kXcd;
  const int q = total / kXcd, r = total % kXcd;
  return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

// Storage types of the conv tensors (se_conv2d_desc.dtype, SE_DTYPE_*): element
// type, a load as float and a round-to-nearest-even store at an element index,
// and a raw buffer load of one element at byte offsets (as float).
template <int SD> struct Stor { typedef float T; };
template <> struct Stor<1> { typedef __bf16 T; };
template <> struct Stor<2> { typedef _Float16 T; };
template <int SD> __device__ __forceinline__ float ld_s(const void* p, long long i) {
  return (float)static_cast<const typename Stor<SD>::T*>(p)[i];
}
template <int SD> __device__ __forceinline__ void st_s(void* p, long long i, float v) {
  static_cast<typename Stor<SD>::T*>(p)[i] = (typename Stor<SD>::T)v;
}
template <int SD> __device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  if constexpr (SD == 0) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  } else {
    const unsigned short v = __builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0);
    if constexpr (SD == 1) return __builtin_bit_cast(float, (unsigned)v << 16);
    else return (float)__builtin_bit_cast(_Float16, v);
  }
}
// Raw bits of one 16-bit storage element (zero-extended), for the one-term split kernels
// whose MFMA format is the storage format (bf16 storage + SE_MATH_BF16, fp16 + SE_MATH_F16):
// the element is already its own hi operand, so it is staged as loaded and packed pairwise
// into LDS, with no convert in between (a convert right behind each load made the compiler
// wait for every load in turn: 2-2.5x slower gathers than the fp32-storage form).
template <int SD> struct StageT { typedef unsigned T; };
template <> struct StageT<0> { typedef float T; };
__device__ __forceinline__ unsigned bload_raw16(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0);
}
__device__ __forceinline__ unsigned ld_raw16(const void* p, long long i) {
  return static_cast<const unsigned short*>(p)[i];
}
// a load of element i of a tensor of runtime storage type sd (small prologue kernels)
__device__ __forceinline__ float ld_any(const void* p, long long i, int sd) {
  return sd == 1 ? ld_s<1>(p, i) : (sd == 2 ? ld_s<2>(p, i) : ld_s<0>(p, i));
}
__device__ __forceinline__ void st_any(void* p, long long i, float v, int sd) {
  if (sd == 1) st_s<1>(p, i, v); else if (sd == 2) st_s<2>(p, i, v); else st_s<0>(p, i, v);
}

struct GatherArgs {
  const float* X;      // gathered tensor [B, Cg, Hi, Wi] (fp32, or 16-bit: see SD)
  const int4* ktab;    // [Kp] {c*Hi*Wi + offh*Wi + offw, offh, offw, 0}
  const float* Wp;     // [Kp, ldw]
  const float* bias;   // [N] or nullptr
  const float* zero;   // zeroed workspace page
  float* Y;            // [B, N, Ho, Wo]
  int Cg, Hi, Wi;
  int N, Ho, Wo;
  int ph, pw, Sh, Sw, Qh, Qw, sh, sw;
  int Kp, ldw, M;
  // FRCRN decoder skip join folded into the GEMM (se_conv2d_*_joined,
  // frcrn.py:93-101): the joined tensor complex_concat([align(x), s]) has the
  // channel chunks [x_re, s_re, x_im, s_im] of jh channels each and is never
  // materialised. Gather side (jh > 0): X holds s (grid Hi x Wi, 2*jh channels
  // per batch item), X2 holds x on its own grid H2 x W2 (rows >= H2 read as 0:
  // F.pad; columns >= Wi are never read: x[..., :-1]).
  const float* X2;
  int jh, H2, W2;
  int jcat;            // join order: 0 complex_concat [x_re, s_re, x_im, s_im], 1 torch.cat [x, s]
  // Output side (yjh > 0, data-grad): the chunks of Y go to Y (s chunks, grid
  // Ho x Wo) and Y2 (x chunks, grid YH2 x YW2; rows >= YH2 are dropped).
  float* Y2;
  int yjh, YH2, YW2;
  // SE_MATH_F16X3: device max |.| of the gathered tensor(s) and of the weights
  const float* amax_a;
  const float* amax_w;
  // gather_stencil_kernel: per-tap input offsets, read as scalars from the kernel
  // arguments
  int ntaps;
  int toffh[kMaxTaps], toffw[kMaxTaps];
};

// LDS images of both operands are column-interleaved inside every 64-wide
// wave block: column 32*i + l is stored at 2*l + i, so each lane fetches its
// two MFMA operands (i = 0, 1) with one conflict-free ds_read_b64. The weight
// columns are pre-interleaved by prep_class_kernel (ldw >= 64).
__device__ __forceinline__ int ilv64(int c) { return (c & ~63) | ((c & 31) << 1) | ((c >> 5) & 1); }

// TU ("tap-uniform"): every K-step lies inside one tap (Cg % kBK == 0), so a
// lane's bounds check and 32-bit voffset are computed once per step and the
// 16 channel loads are raw buffer loads with a scalar soffset = c*Hi*Wi*4;
// out-of-range lanes get an out-of-bounds voffset and the hardware returns 0.
template <int BN, int BM, int WN, int WM, bool TU>
__global__ void __launch_bounds__(kThreads, 2)   // 2 waves/SIMD: <= 256 VGPR+AGPR
gather_gemm_kernel(const GatherArgs a) {
  static_assert(WN * WM == 4, "4 waves");
  constexpr int TN = BN / WN, TM = BM / WM;       // wave tile
  constexpr int RN = TN / 32, RM = TM / 32;       // 32x32 MFMA repeats
  static_assert(RN == 2 && RM == 2, "interleaved LDS images assume 64-wide wave tiles");
  constexpr int KR = kThreads / BM;               // threads per m column
  constexpr int AJ = kBK / KR;                    // A rows per thread per step
  constexpr int WV = (kBK * BN) / (4 * kThreads); // float4 weight loads/thread
  static_assert(KR >= 1 && WV >= 1, "tile shape");

  __shared__ __attribute__((aligned(16))) float sA[2][kBK][BM];
  __shared__ __attribute__((aligned(16))) float sW[2][kBK][BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  // logical tile: N-tiles of one M-tile adjacent, consecutive M-tiles on one XCD
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int m0 = (tile / gridDim.y) * BM, n0 = (tile % gridDim.y) * BN;
  const long long HiWi = (long long)a.Hi * a.Wi;

  // --- this thread's gather column (fixed for the whole K loop) ---
  const int am = tid % BM;
  const int am_pos = ilv64(am);
  const int akr = __builtin_amdgcn_readfirstlane(tid / BM);   // wave-uniform k row
  const int m = m0 + am;
  const bool mval = m < a.M;
  int hb = 0, wb = 0;
  long long xbase = 0;
  if (mval) {
    const int qhw = a.Qh * a.Qw;
    const int b = m / qhw, r = m - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    hb = qh * a.sh;
    wb = qw * a.sw;
    xbase = (long long)b * a.Cg * HiWi + (long long)hb * a.Wi + wb;
  }

  // two register staging sets: tile t+2 is loading while tile t+1 waits to be
  // written to LDS and tile t is consumed by the MFMAs (prefetch distance 2)
  struct Stage { float ra[AJ]; f32x4 rw[WV]; };
  Stage s0, s1;
  // TU path: buffer descriptors built from wave-uniform values only
  const int b0 = m0 / (a.Qh * a.Qw);               // first batch item of the tile
  using se::uniform_ptr;   // descriptor inputs made provably uniform
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.X + (long long)b0 * a.Cg * HiWi), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rwp = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(a.Wp), (short)0, 0x7FFFFFFF, 0x00020000);
  int xoff = 0, woff[WV];
  if constexpr (TU) {
    const int qhw = a.Qh * a.Qw;
    if (mval) {
      const int b = m / qhw;
      xoff = (int)(((long long)(b - b0) * a.Cg * HiWi + (long long)hb * a.Wi + wb) * 4);
    }
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int idx = tid + kThreads * j;
      const int kr = idx / (BN / 4), c4 = idx % (BN / 4);
      woff[j] = (kr * a.ldw + n0 + 4 * c4) * 4;
    }
  }
  auto load_tile = [&](Stage& st, int k0) __attribute__((always_inline)) {
    if constexpr (TU) {
      const int4 e0 = a.ktab[k0];                     // tap of this step (uniform)
      const int tap = k0 / a.Cg;
      const int c0 = k0 - tap * a.Cg + akr;
      const int hi = hb + e0.y, wi = wb + e0.z;
      const bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      const int vo = ok ? xoff + (e0.y * a.Wi + e0.z) * 4 : (int)0x80000000;
      const int cs = (int)(HiWi * 4);
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        st.ra[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo, (c0 + KR * j) * cs, 0));
      const int so = k0 * a.ldw * 4;
#pragma unroll
      for (int j = 0; j < WV; ++j)
        st.rw[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rwp, woff[j], so, 0));
      return;
    }
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int4 e = a.ktab[k0 + akr + KR * j];        // uniform index -> s_load
      const int hi = hb + e.y, wi = wb + e.z;
      const bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      // unconditional load (a predicated one makes hipcc branch around it and
      // drain vmcnt(0) per element); invalid lanes read the zero page
      st.ra[j] = *(ok ? a.X + xbase + e.x : a.zero);
    }
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int idx = tid + kThreads * j;           // float4 index in [BK][BN/4]
      const int kr = idx / (BN / 4), c4 = idx % (BN / 4);
      st.rw[j] = *reinterpret_cast<const f32x4*>(a.Wp + (long long)(k0 + kr) * a.ldw + n0 + 4 * c4);
    }
  };
  auto store_tile = [&](const Stage& st, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) sA[buf][akr + KR * j][am_pos] = st.ra[j];
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int idx = tid + kThreads * j;
      const int kr = idx / (BN / 4), c4 = idx % (BN / 4);
      *reinterpret_cast<f32x4*>(&sW[buf][kr][4 * c4]) = st.rw[j];
    }
  };

  f32x16 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lk = lane >> 5, lc = lane & 31;
  const int wcol = wn * TN + 2 * lc, mcol = wm * TM + 2 * lc;
  // one K-step of MFMAs on LDS buffer `cur`
  auto compute = [&](int cur) __attribute__((always_inline)) {
    // Fragments of the whole step in registers, fetched in two halves: the
    // second half's ds_reads are issued (and fenced) before the first half's
    // MFMAs, so the LDS latency hides under 32 MFMAs instead of stalling each.
    constexpr int KP = kBK / 2, H = KP / 2;
    f32x2 fa[KP], fb[KP];
#pragma unroll
    for (int kk = 0; kk < H; ++kk) {
      fa[kk] = *reinterpret_cast<const f32x2*>(&sW[cur][2 * kk + lk][wcol]);
      fb[kk] = *reinterpret_cast<const f32x2*>(&sA[cur][2 * kk + lk][mcol]);
    }
#pragma unroll
    for (int kk = H; kk < KP; ++kk) {
      fa[kk] = *reinterpret_cast<const f32x2*>(&sW[cur][2 * kk + lk][wcol]);
      fb[kk] = *reinterpret_cast<const f32x2*>(&sA[cur][2 * kk + lk][mcol]);
    }
#pragma unroll
    for (int kk = 0; kk < KP; ++kk) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk].x, fb[kk].x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk].x, fb[kk].y, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk].y, fb[kk].x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk].y, fb[kk].y, acc[1][1], 0, 0, 0);
    }
  };
  // the step's non-MFMA stream (next tiles' loads, fragment reads,
  // LDS writes) interleaved into the 64-cycle MFMA gaps
  auto interleave = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                  // first fragments
#pragma unroll
    for (int i = 0; i < 4 * (kBK / 2); ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                // MFMA
      __builtin_amdgcn_sched_group_barrier(0x080, 1, 0);                // DS
      if (i % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // global load
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);                // VALU
    }
  };

  const int nk = a.Kp / kBK;
  // prologue: tile 0 -> LDS[0]; tile 1 in flight in s1
  load_tile(s0, 0);
  store_tile(s0, 0);
  if (nk > 1) load_tile(s1, kBK);
  __syncthreads();
  // main loop, unrolled by two so the staging sets alternate by name
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    // unconditional (clamped) loads / stores: one scheduling region per step;
    // a clamped reload of the last tile lands in the buffer no step reads
    load_tile(s0, min(kt + 2, nk - 1) * kBK);
    compute(0);
    store_tile(s1, 1);
    interleave();
    __syncthreads();
    load_tile(s1, min(kt + 3, nk - 1) * kBK);
    compute(1);
    store_tile(s0, 0);
    interleave();
    __syncthreads();
  }
  if (kt < nk) compute(0);   // odd tile count: the last tile sits in LDS[0]

  // --- epilogue: lane -> m (coalesced along time), registers -> n ---
  __syncthreads();                                 // every wave is done reading LDS[0]
  float* sBias = &sW[0][0][0];                     // reuse the drained weight tile
  for (int i = tid; i < BN; i += kThreads) {
    const int n = n0 + i;
    sBias[i] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
  }
  __syncthreads();
  const long long HoWo = (long long)a.Ho * a.Wo;
  const bool full_n = n0 + BN <= a.N;
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const int mm = m0 + wm * TM + 32 * j + lc;
    if (mm >= a.M) continue;
    const int qhw = a.Qh * a.Qw;
    const int b = mm / qhw, r = mm - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    const int nl0 = wn * TN + 4 * lk;               // this lane's first local row
    float* yb = a.Y + (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo +
                (a.pw + a.Sw * qw) + (long long)(n0 + nl0) * HoWo;
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        const int nl = 32 * i + (r2 & 3) + 8 * (r2 >> 2);   // compile-time
        if (full_n || n0 + nl0 + nl < a.N) yb[(long long)nl * HoWo] = acc[i][j][r2] + sBias[nl0 + nl];
      }
  }
}

// Small-N variant (N <= 16: final_conv 128->2, the CCBAM k7 conv 4->2 and its
// data-grad): HBM-bound, one output position per thread, weights in LDS.
template <int NOUT, int SD = 0>
__global__ void __launch_bounds__(kThreads)
gather_smalln_kernel(const GatherArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sWs[];  // [Kp][NOUT]
  for (int i = threadIdx.x; i < a.Kp * NOUT; i += kThreads) {
    const int k = i / NOUT, n = i % NOUT;
    sWs[i] = a.Wp[(long long)k * a.ldw + n];
  }
  __syncthreads();
  const int m = blockIdx.x * kThreads + threadIdx.x;
  if (m >= a.M) return;
  const int qhw = a.Qh * a.Qw;
  const int b = m / qhw, r = m - b * qhw;
  const int qh = r / a.Qw, qw = r - qh * a.Qw;
  const int hb = qh * a.sh, wb = qw * a.sw;
  const long long HiWi = (long long)a.Hi * a.Wi;
  const long long xbase = (long long)b * a.Cg * HiWi + (long long)hb * a.Wi + wb;
  float acc[NOUT];
#pragma unroll
  for (int n = 0; n < NOUT; ++n) acc[n] = 0.f;
#pragma unroll 8
  for (int k = 0; k < a.Kp; ++k) {     // Kp % 32 == 0: eight gathered loads in flight
    const int4 e = a.ktab[k];
    const int hi = hb + e.y, wi = wb + e.z;
    const bool ok = (unsigned)hi < (unsigned)a.Hi && (unsigned)wi < (unsigned)a.Wi;
    const float xv = ld_s<SD>(a.X, ok ? xbase + e.x : 0);
    const float x = ok ? xv : 0.f;
#pragma unroll
    for (int n = 0; n < NOUT; ++n) acc[n] = fmaf(x, sWs[k * NOUT + n], acc[n]);
  }
  const long long HoWo = (long long)a.Ho * a.Wo;
  const long long ybase = (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo +
                          (a.pw + a.Sw * qw);
#pragma unroll
  for (int n = 0; n < NOUT; ++n)
    if (n < a.N) st_s<SD>(a.Y, ybase + n * HoWo, acc[n] + (a.bias ? a.bias[n] : 0.f));
}

// Small-N stride-1 conv as an LDS stencil (CCBAM's spatial ComplexConv2d(4 -> 2, k7,
// pad 3) and its data-grad, ccbam.py:65-86): a workgroup stages a CG x (32 + halo)
// x (64 + halo) input tile once, and each thread forms kStR output rows of one
// column from it, so a gathered element is loaded from HBM / L2 once per tile instead
// of once per tap. Per output the products are added in gather_smalln_kernel's order
// (k = tap * CG + c, fmaf), so the results are bit-identical to it. The weights of a
// k are uniform (scalar loads); tap offsets come from the kernel arguments.
constexpr int kStW = 64, kStRG = 4, kStR = 8;   // tile: 64 columns x (4 x 8) rows
template <int NOUT, int CG>
__global__ void __launch_bounds__(kThreads)
gather_stencil_kernel(const GatherArgs a, int h0, int w0, int th, int tw) {
  extern __shared__ float sx[];   // [CG][th][tw]
  const int b = blockIdx.z;
  const int qh0 = blockIdx.y * (kStRG * kStR), qw0 = blockIdx.x * kStW;
  const long long HiWi = (long long)a.Hi * a.Wi;
  const float* xb = a.X + (long long)b * CG * HiWi;
  const int plane = th * tw;
  for (int i = threadIdx.x; i < CG * plane; i += kThreads) {
    const int c = i / plane, rr = i - c * plane;
    const int r = rr / tw, col = rr - r * tw;
    const int hi = qh0 + h0 + r, wi = qw0 + w0 + col;
    sx[i] = ((unsigned)hi < (unsigned)a.Hi && (unsigned)wi < (unsigned)a.Wi)
                ? xb[(long long)c * HiWi + (long long)hi * a.Wi + wi] : 0.f;
  }
  __syncthreads();
  const int lc = threadIdx.x & 63, r0 = (threadIdx.x >> 6) * kStR;
  float acc[kStR][NOUT];
#pragma unroll
  for (int r = 0; r < kStR; ++r)
#pragma unroll
    for (int n = 0; n < NOUT; ++n) acc[r][n] = 0.f;
  for (int t = 0; t < a.ntaps; ++t) {
    const int base = (r0 + a.toffh[t] - h0) * tw + lc + a.toffw[t] - w0;
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      const float* wk = a.Wp + (long long)(t * CG + c) * a.ldw;
      float w[NOUT];
#pragma unroll
      for (int n = 0; n < NOUT; ++n) w[n] = wk[n];
      const float* src = sx + c * plane + base;
#pragma unroll
      for (int r = 0; r < kStR; ++r) {
        const float v = src[r * tw];
#pragma unroll
        for (int n = 0; n < NOUT; ++n) acc[r][n] = fmaf(v, w[n], acc[r][n]);
      }
    }
  }
  const long long HoWo = (long long)a.Ho * a.Wo;
  const int qw = qw0 + lc;
  if (qw >= a.Qw) return;
#pragma unroll
  for (int r = 0; r < kStR; ++r) {
    const int qh = qh0 + r0 + r;
    if (qh >= a.Qh) break;
    const long long yb = (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo + (a.pw + a.Sw * qw);
#pragma unroll
    for (int n = 0; n < NOUT; ++n)
      if (n < a.N) a.Y[yb + n * HoWo] = acc[r][n] + (a.bias ? a.bias[n] : 0.f);
  }
}

// Small-N stride-1 conv over MANY channels as a chunked LDS stencil: DCUNet's final
// ComplexConvTranspose2d (128 -> 2 channels, k (7, 5), stride (2, 2); its four phase
// classes are stride-1 convs of 2-4 x 2-3 taps; _1903_03107_dcunet.py:80-83,
// architectures.py:63-72). A workgroup owns a (kScRows x kStW) output tile of one
// class; per chunk of kScC channels it stages the input tile plus halo in LDS (the
// next chunk's loads are in flight meanwhile), and each thread forms kScR rows of one
// column: per (channel, tap column) it reads the kScR + NTH - 1 input rows its NTH
// row taps touch once and reuses them from registers. The class's row offsets are
// consecutive and descending (offh[a] = offh[0] - a, phase_dim), so the tap-row
// index into that window is a compile-time constant. Weights are uniform (scalar
// loads): Wp[(t * Cg + c) * ldw + n], t = a * ntw + b.
#if SE_STC_DEBUG
// bounds instrumentation of the chunked stencil (debug variant builds only): every
// index is checked against its buffer and clamped into it; violations are counted
// per kind with vector atomics and read back by se_debug_stencil_counts
__device__ int g_stc_dbg[8];
#define STC_CHECK(kind, idx, lim) \
  do { if ((long long)(idx) < 0 || (long long)(idx) >= (long long)(lim)) atomicAdd(&g_stc_dbg[kind], 1); } while (0)
#define STC_CLAMP(idx, lim) (max(0ll, min((long long)(idx), (long long)(lim) - 1)))
#else
#define STC_CHECK(kind, idx, lim) do { } while (0)
#define STC_CLAMP(idx, lim) (idx)
#endif
constexpr int kScC = 8, kScR = 4, kScRows = 4 * kScR;   // 8 channels, 16 x 64 outputs
constexpr int kScPitch = kStW + 8;                        // LDS row: 64 columns + a halo <= 8
template <int NO, int NTH, int SD>
__global__ void __launch_bounds__(kThreads)
gather_stencil_ch_kernel(const GatherArgs a, int h0, int w0, int ntw, int ngrp, int cpg, float* part) {
  constexpr int TH = kScRows + NTH - 1, WIN = kScR + NTH - 1;
  constexpr int tw = kScPitch, plane = TH * tw, chunk = kScC * plane;   // compile-time indexing
  extern __shared__ float sx[];   // [kScC][TH][kScPitch]
  // blockIdx.z = (item, channel group): the group's channels [cg0, cg1)
  const int b = blockIdx.z / ngrp, grp = blockIdx.z - b * ngrp;
  const int cg0 = grp * cpg, cg1 = min(a.Cg, cg0 + cpg);
  const int qh0 = blockIdx.y * kScRows, qw0 = blockIdx.x * kStW;
  constexpr int ES = SD ? 2 : 4;
  const int HiWi = a.Hi * a.Wi;   // the host checks Cg * Hi * Wi * ES < 2^31
  // 32-bit offsets into the item's planes through a buffer resource (out-of-range
  // offset: reads 0); 16-bit elements are staged as raw bits and converted when they
  // are written to LDS, so no convert waits on a load in flight
  // (se::uniform_ptr widens the two words as unsigned: a low word >= 2^31 must not
  // sign-extend into the high half of the base)
  // joined input (a.X2): X holds s (2 jh channels per item, grid Hi x Wi), X2 holds x on its
  // grid H2 x W2 (the F.pad zeros outside, x's extra trailing column never read); torch.cat
  // order [x, s] (DCUNet's decoder join, a.jcat) or complex_concat's [x_re, s_re, x_im, s_im]
  // (DCCRN's / FRCRN's, round 6); a chunk of kScC channels lies in one source (jh % kScC == 0,
  // checked by the host)
  const bool jn = a.X2 != nullptr;
  const int cpb = jn ? 2 * a.jh : a.Cg, H2W2 = a.H2 * a.W2;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      se::uniform_ptr((const char*)a.X + (long long)b * cpb * HiWi * ES), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx2 = jn ? __builtin_amdgcn_make_buffer_rsrc(
      se::uniform_ptr((const char*)a.X2 + (long long)b * cpb * H2W2 * ES), (short)0, 0x7FFFFFFF, 0x00020000) : rx;
  constexpr int PF = (chunk + kThreads - 1) / kThreads;
  typename StageT<SD>::T pf[PF];
  auto fetch = [&](int c0) __attribute__((always_inline)) {
    const int q = jn ? c0 / a.jh : 0;                   // the chunk's join block (chunk-uniform)
    const bool from_x = jn && (a.jcat ? q < 2 : (q & 1) == 0);
    // the chunk's first channel in its source
    const int cs = !jn ? c0 : a.jcat ? (from_x ? c0 : c0 - cpb) : (q >> 1) * a.jh + (c0 - q * a.jh);
    // x is addressed on its own grid (row pitch W2) but bounded by the joined grid: its columns
    // past Wi are the frame complex_concat's alignment crops (x[..., :-1]), read as zeros
    const int sh = from_x ? min(a.H2, a.Hi) : a.Hi, sw = from_x ? min(a.W2, a.Wi) : a.Wi;
    const int spl = from_x ? H2W2 : HiWi, pitch = from_x ? a.W2 : a.Wi;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int i = threadIdx.x + j * kThreads;
      const int c = i / plane, rr = i - c * plane;
      const int r = rr / tw, col = rr - r * tw;
      const int hi = qh0 + h0 + r, wi = qw0 + w0 + col;
      const bool ok = (chunk % kThreads == 0 || i < chunk) && c0 + c < cg1 && (unsigned)hi < (unsigned)sh && (unsigned)wi < (unsigned)sw;
      const int vo = ok ? ((cs + c) * spl + hi * pitch + wi) * ES : (int)0x80000000;
      if (ok) STC_CHECK(0, vo, (long long)(jn ? cpb : a.Cg) * spl * ES);
      if constexpr (SD == 0) pf[j] = bload<0>(from_x ? rx2 : rx, vo, 0);
      else pf[j] = bload_raw16(from_x ? rx2 : rx, vo, 0);
    }
  };
  auto to_f32 = [](typename StageT<SD>::T v) __attribute__((always_inline)) {
    if constexpr (SD == 0) return v;
    else if constexpr (SD == 1) return __builtin_bit_cast(float, v << 16);
    else return (float)__builtin_bit_cast(_Float16, (unsigned short)v);
  };
  const int lc = threadIdx.x & 63, r0 = (threadIdx.x >> 6) * kScR;
  float acc[kScR][NO];
#pragma unroll
  for (int r = 0; r < kScR; ++r)
#pragma unroll
    for (int n = 0; n < NO; ++n) acc[r][n] = 0.f;
  fetch(cg0);
  for (int c0 = cg0; c0 < cg1; c0 += kScC) {
    __syncthreads();   // the previous chunk is consumed
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int i = threadIdx.x + j * kThreads;
      if (chunk % kThreads == 0 || i < chunk) { STC_CHECK(1, i, chunk); sx[STC_CLAMP(i, chunk)] = to_f32(pf[j]); }
    }
    __syncthreads();
    if (c0 + kScC < cg1) fetch(c0 + kScC);
    const int nc = min(kScC, cg1 - c0);
    for (int c = 0; c < nc; ++c) {
      for (int bw = 0; bw < ntw; ++bw) {
        const int sbase = c * plane + r0 * tw + lc + a.toffw[bw] - w0;
        float v[WIN];
#pragma unroll
        for (int i = 0; i < WIN; ++i) { STC_CHECK(2, sbase + i * tw, chunk); v[i] = sx[STC_CLAMP(sbase + i * tw, chunk)]; }
#pragma unroll
        for (int ah = 0; ah < NTH; ++ah) {
          const long long wo = (long long)((ah * ntw + bw) * a.Cg + c0 + c) * a.ldw;
          STC_CHECK(3, wo + NO - 1, (long long)a.Kp * a.ldw);
          const float* wk = a.Wp + STC_CLAMP(wo, (long long)a.Kp * a.ldw - NO + 1);
          float w[NO];
#pragma unroll
          for (int n = 0; n < NO; ++n) w[n] = wk[n];
#pragma unroll
          for (int r = 0; r < kScR; ++r)
#pragma unroll
            for (int n = 0; n < NO; ++n) acc[r][n] = fmaf(v[r + NTH - 1 - ah], w[n], acc[r][n]);
        }
      }
    }
  }
  const long long HoWo = (long long)a.Ho * a.Wo, QQ = (long long)a.Qh * a.Qw;
  const int qw = qw0 + lc;
  if (qw >= a.Qw) return;
#pragma unroll
  for (int r = 0; r < kScR; ++r) {
    const int qh = qh0 + r0 + r;
    if (qh >= a.Qh) break;
    if (part) {   // channel groups: this group's partial sums, [grp][b][n][qh][qw]
      const long long pb = ((long long)grp * (gridDim.z / ngrp) + b) * a.N * QQ + (long long)qh * a.Qw + qw;
#pragma unroll
      for (int n = 0; n < NO; ++n)
        if (n < a.N) { STC_CHECK(4, pb + n * QQ, (long long)gridDim.z * a.N * QQ); part[STC_CLAMP(pb + n * QQ, (long long)gridDim.z * a.N * QQ)] = acc[r][n]; }
      continue;
    }
    const long long yb = (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo + (a.pw + a.Sw * qw);
#pragma unroll
    for (int n = 0; n < NO; ++n)
      if (n < a.N) {
        STC_CHECK(5, yb + n * HoWo, (long long)(gridDim.z / ngrp) * a.N * HoWo);
        st_s<SD>(a.Y, STC_CLAMP(yb + n * HoWo, (long long)(gridDim.z / ngrp) * a.N * HoWo), acc[r][n] + (a.bias ? a.bias[n] : 0.f));
      }
  }
}

#if SE_STC_DEBUG
extern "C" int se_debug_stencil_counts(int* out8) {
  return hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stc_dbg), 8 * sizeof(int)) == hipSuccess ? 0 : -1;
}
#endif

// Y at the class's positions = bias + the channel groups' partial sums, added in group
// order (deterministic). grid ceil(B * N * Qh * Qw / 256)
template <int SD>
__global__ void __launch_bounds__(kThreads)
stencil_ch_reduce_kernel(const GatherArgs a, int ngrp, const float* __restrict__ part) {
  const long long QQ = (long long)a.Qh * a.Qw, per = (long long)(a.M / QQ) * a.N * QQ;
  const long long i = blockIdx.x * (long long)kThreads + threadIdx.x;
  if (i >= per) return;
  float v = 0.f;
  for (int gi = 0; gi < ngrp; ++gi) v += part[gi * per + i];
  const long long bn = i / QQ, r = i - bn * QQ;
  const int n = (int)(bn % a.N);
  const int qh = (int)(r / a.Qw), qw = (int)(r - (long long)qh * a.Qw);
  const long long HoWo = (long long)a.Ho * a.Wo;
  st_s<SD>(a.Y, bn * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo + (a.pw + a.Sw * qw), v + (a.bias ? a.bias[n] : 0.f));
}

// ---------------------------------------------------------------------------
// Weight-grad reduction GEMM: dWp[k, n] = sum_m G[m, k] * D[m, n]
// Each workgroup reduces one m-range (split) for one BKO x BNO tile and
// writes a partial slab; wgrad_finish_kernel sums the slabs (deterministic).
// ---------------------------------------------------------------------------
struct WgradArgs {
  const float* X;      // gathered tensor [B, Cg, Hi, Wi]
  const int4* ktab;    // [Kp]
  const float* D;      // direct tensor [B, N, Qh, Qw]
  const float* zero;   // zeroed workspace page
  float* slab;         // [splits, Kp, Np]
  int Cg, Hi, Wi;
  int N, Qh, Qw, sh, sw;
  int Kp, Np, M;
  int m_per_split;     // multiple of the kernel's BMR (64)
  // joined D (transposed conv over the decoder skip join, see GatherArgs):
  // D holds s (2*djh channels, grid Qh x Qw), D2 holds x on DH2 x DW2.
  const float* D2;
  int djh, DH2, DW2;
  int djcat;           // join order (GatherArgs::jcat)
  // SE_MATH_F16X3: device max |.| of G (the gathered tensor) and of D (both sources)
  const float* amax_g;
  const float* amax_d;
  // per-tap input offsets (wgrad_ktab)
  int toffh[kMaxTaps], toffw[kMaxTaps];
  // wgrad_x3_kernel: tile space (k-tiles, n-tiles, m-splits) walked by its 1-D grid
  int vk, vn, vs;
  // wgrad_x3_kernel with ktab == nullptr: entries computed in the kernel from
  // (ntaps, toffh, toffw), k = t * Cg + c (as prep_class_kernel)
  int ntaps;
};

// ktab[k] of a weight-grad pass (prep_class_kernel's rule) from the tap table
__device__ __forceinline__ int4 wgrad_ktab(const WgradArgs& a, int k) {
  int4 e;
  if (k < a.ntaps * a.Cg) {
    const int t = k / a.Cg, c = k - t * a.Cg;
    e.x = (int)((long long)c * a.Hi * a.Wi + (long long)a.toffh[t] * a.Wi + a.toffw[t]);
    e.y = a.toffh[t];
    e.z = a.toffw[t];
  } else {
    e.x = 0; e.y = kInvalidOff; e.z = 0;
  }
  e.w = 0;
  return e;
}

// Small-N weight grad (N <= 8: FRCRN's final_conv 128->2 and the CCBAM spatial
// ComplexConv2d 4->2): an MFMA tile would be >= 75% padding, and the pass is
// bound by reading the gathered tensor once. One workgroup = KG rows of K x
// one m-split; a thread walks positions m (coalesced along time), keeps its
// N values of D in registers and accumulates KG*N products; the block then
// reduces and writes one slab row block (same slab / finish path as the GEMM).
template <int NOUT>
__global__ void __launch_bounds__(kThreads)
wgrad_smalln_kernel(const WgradArgs a) {
  constexpr int KG = 16;
  const int k0 = blockIdx.x * KG, split = blockIdx.y;
  const int mbeg = split * a.m_per_split, mend = min(a.M, mbeg + a.m_per_split);
  const int QQ = a.Qh * a.Qw;
  const long long HiWi = (long long)a.Hi * a.Wi;
  int4 e[KG];
#pragma unroll
  for (int k = 0; k < KG; ++k) e[k] = a.ktab[k0 + k];
  float acc[KG][NOUT];
#pragma unroll
  for (int k = 0; k < KG; ++k)
#pragma unroll
    for (int n = 0; n < NOUT; ++n) acc[k][n] = 0.f;
  // position m -> (b, qh, qw), advanced incrementally by kThreads per step
  int m = mbeg + threadIdx.x;
  int b = m / QQ, r = m - b * QQ;
  int qh = r / a.Qw, qw = r - qh * a.Qw;
  for (; m < mend; m += kThreads) {
    const int hb = qh * a.sh, wb = qw * a.sw;
    float dv[NOUT];
#pragma unroll
    for (int n = 0; n < NOUT; ++n)
      dv[n] = n < a.N ? a.D[(((long long)b * a.N + n) * a.Qh + qh) * a.Qw + qw] : 0.f;
    const long long xbase = (long long)b * a.Cg * HiWi + (long long)hb * a.Wi + wb;
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int hi = hb + e[k].y, wi = wb + e[k].z;
      const bool ok = (unsigned)hi < (unsigned)a.Hi && (unsigned)wi < (unsigned)a.Wi;
      const float xv = a.X[ok ? xbase + e[k].x : 0];
      const float x = ok ? xv : 0.f;
#pragma unroll
      for (int n = 0; n < NOUT; ++n) acc[k][n] = fmaf(x, dv[n], acc[k][n]);
    }
    qw += kThreads;
    while (qw >= a.Qw) {
      qw -= a.Qw;
      if (++qh == a.Qh) { qh = 0; ++b; }
    }
  }
  __shared__ float red[kThreads / 64][KG * NOUT];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < KG; ++k)
#pragma unroll
    for (int n = 0; n < NOUT; ++n) {
      const float v = se::wave_sum(acc[k][n]);
      if (lane == 0) red[w][k * NOUT + n] = v;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < KG * NOUT; i += kThreads) {
    const float v = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    a.slab[((long long)split * a.Kp + k0 + i / NOUT) * a.Np + (i % NOUT)] = v;
  }
}

// One reduction step covers BMR consecutive positions m; a wave-instruction
// loads LPW = 64 / BMR rows (k or n) x BMR positions, lanes along m so every
// load is coalesced along the time axis.
// TU: the K-tile lies inside one tap (Cg % BKO == 0): per step a lane's bounds
// check and 32-bit voffsets are computed once, rows are scalar soffsets.
template <int BKO, int BNO, int WK, int WNn, int BMR, bool TU>
__global__ void __launch_bounds__(kThreads)
wgrad_gemm_kernel(const WgradArgs a) {
  static_assert(WK * WNn == 4, "4 waves");
  constexpr int TK = BKO / WK, TN = BNO / WNn;
  constexpr int RK = TK / 32, RN = TN / 32;
  constexpr int LPW = 64 / BMR;            // rows per wave-instruction
  constexpr int RS = 4 * LPW;              // rows covered by the workgroup per j
  constexpr int GJ = BKO / RS, DJ = BNO / RS;
  constexpr int L = BMR + 2;               // padded [row][m] images (even: 8-B aligned rows)
  __shared__ __attribute__((aligned(16))) float sG[2][BKO * L];
  __shared__ __attribute__((aligned(16))) float sD[2][BNO * L];
  __shared__ int4 sK[BKO];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave / WNn, wnn = wave % WNn;
  // logical tile: every (k, n) tile of one m-split adjacent (they share D rows)
  const int nkn = gridDim.x * gridDim.y;
  const int tile = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, nkn * gridDim.z);
  const int split = tile / nkn, kn = tile % nkn;
  const int k0 = (kn % gridDim.x) * BKO, n0 = (kn / gridDim.x) * BNO;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const long long HiWi = (long long)a.Hi * a.Wi;
  const long long QQ = (long long)a.Qh * a.Qw;
  const int ml = lane % BMR, lr = lane / BMR;
  const int row0 = wave * LPW + lr;        // + RS * j

  for (int i = tid; i < BKO; i += kThreads) sK[i] = a.ktab[k0 + i];
  __syncthreads();

  // incremental decode of this lane's m = mbeg + ml + step*BMR
  int cb, cqh, cqw;
  {
    const long long mm = mbeg + ml;
    cb = (int)(mm / QQ);
    const int r = (int)(mm - cb * QQ);
    cqh = r / a.Qw;
    cqw = r - cqh * a.Qw;
  }
  struct Stage { float rg[GJ], rd[DJ]; };
  Stage st0, st1;   // two register staging sets: prefetch distance 2
  // TU buffer descriptors over the split's first batch item (uniform inputs)
  using se::uniform_ptr;
  const int bfirst = (int)(mbeg / QQ);
  __amdgpu_buffer_rsrc_t rg_src = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.X + (long long)bfirst * a.Cg * HiWi), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rd_src = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.D + (long long)bfirst * a.N * QQ), (short)0, 0x7FFFFFFF, 0x00020000);
  const int4 tap_e = a.ktab[k0];              // TU: the tile's single tap
  const int cbase = k0 % a.Cg;
  // m += BMR in (b, qh, qw), branch-free (a data-dependent loop here would split
  // the step into separate scheduling regions): one wrap when Qw >= BMR,
  // otherwise by division (uniform, loop-invariant choice)
  const bool one_wrap = a.Qw >= BMR;
  auto advance = [&]() __attribute__((always_inline)) {
    if (one_wrap) {
      cqw += BMR;
      const bool w1 = cqw >= a.Qw;
      cqw -= w1 ? a.Qw : 0;
      cqh += w1 ? 1 : 0;
      const bool w2 = cqh >= a.Qh;
      cqh = w2 ? 0 : cqh;
      cb += w2 ? 1 : 0;
    } else {
      const int t = cqw + BMR;
      const int dq = t / a.Qw;
      cqw = t - dq * a.Qw;
      const int u = cqh + dq;
      const int db = u / a.Qh;
      cqh = u - db * a.Qh;
      cb += db;
    }
  };
  auto load_step = [&](Stage& S, int mstep) __attribute__((always_inline)) {
    if constexpr (TU) {
      const bool mv = mstep + ml < mend;
      const int hi = cqh * a.sh + tap_e.y, wi = cqw * a.sw + tap_e.z;
      const bool ok = mv & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      const int rb = cb - bfirst;
      const int vg = ok ? (int)(((long long)rb * a.Cg * HiWi + (long long)(cbase + lr) * HiWi +
                                 (long long)hi * a.Wi + wi) * 4) : (int)0x80000000;
      const int vd = mv ? (int)(((long long)rb * a.N * QQ + (long long)(n0 + lr) * QQ +
                                 (long long)cqh * a.Qw + cqw) * 4) : (int)0x80000000;
      const int gs = (int)(HiWi * 4), ds = (int)(QQ * 4);
#pragma unroll
      for (int j = 0; j < GJ; ++j)
        S.rg[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            rg_src, vg, (wave * LPW + RS * j) * gs, 0));
#pragma unroll
      for (int j = 0; j < DJ; ++j) {
        const bool nok = n0 + wave * LPW + RS * j + lr < a.N;   // only the Np-padded tail fails
        S.rd[j] = nok ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                          rd_src, vd, (wave * LPW + RS * j) * ds, 0)) : 0.f;
      }
      advance();
      return;
    }
    const bool mv = mstep + ml < mend;
    const int hb = cqh * a.sh, wb = cqw * a.sw;
    const long long xb = (long long)cb * a.Cg * HiWi + (long long)hb * a.Wi + wb;
#pragma unroll
    for (int j = 0; j < GJ; ++j) {
      const int4 e = sK[row0 + RS * j];
      const int hi = hb + e.y, wi = wb + e.z;
      const bool ok = mv & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      S.rg[j] = *(ok ? a.X + xb + e.x : a.zero);
    }
    const long long db = (long long)cb * a.N * QQ + (long long)cqh * a.Qw + cqw;
#pragma unroll
    for (int j = 0; j < DJ; ++j) {
      const int n = n0 + row0 + RS * j;
      const bool ok = mv & (n < a.N);
      S.rd[j] = *(ok ? a.D + db + (long long)n * QQ : a.zero);
    }
    advance();
  };
  auto store_step = [&](const Stage& S, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < GJ; ++j) sG[buf][(row0 + RS * j) * L + ml] = S.rg[j];
#pragma unroll
    for (int j = 0; j < DJ; ++j) sD[buf][(row0 + RS * j) * L + ml] = S.rd[j];
  };

  f32x16 acc[RK][RN];
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nsteps = (mend > mbeg) ? (mend - mbeg + BMR - 1) / BMR : 0;
  const int lk = lane >> 5, lc = lane & 31;
  // one step: MFMAs over LDS[cur]
  auto compute = [&](int cur) __attribute__((always_inline)) {
    // Reduction index of MFMA kk (0..BMR/2-1) for lane half lk is m = kk + (BMR/2)*lk,
    // so k-pairs 2q and 2q+1 of one operand row come from ONE ds_read_b64. The
    // step's fragments are fetched in two fenced halves (second half's reads
    // overlap the first half's MFMAs).
    constexpr int Q = BMR / 4, HQ = Q / 2;
    f32x2 ga[RK][Q], gb[RN][Q];
    const int col = (BMR / 2) * lk;
#pragma unroll
    for (int q = 0; q < HQ; ++q) {
#pragma unroll
      for (int i = 0; i < RK; ++i)
        ga[i][q] = *reinterpret_cast<const f32x2*>(&sG[cur][(wk * TK + 32 * i + lc) * L + col + 2 * q]);
#pragma unroll
      for (int j = 0; j < RN; ++j)
        gb[j][q] = *reinterpret_cast<const f32x2*>(&sD[cur][(wnn * TN + 32 * j + lc) * L + col + 2 * q]);
    }
#pragma unroll
    for (int q = HQ; q < Q; ++q) {
#pragma unroll
      for (int i = 0; i < RK; ++i)
        ga[i][q] = *reinterpret_cast<const f32x2*>(&sG[cur][(wk * TK + 32 * i + lc) * L + col + 2 * q]);
#pragma unroll
      for (int j = 0; j < RN; ++j)
        gb[j][q] = *reinterpret_cast<const f32x2*>(&sD[cur][(wnn * TN + 32 * j + lc) * L + col + 2 * q]);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int i = 0; i < RK; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(e ? ga[i][q].y : ga[i][q].x,
                                                             e ? gb[j][q].y : gb[j][q].x, acc[i][j], 0, 0, 0);
    }
  };
  // one scheduling region per step (loads of step s+2, fragment
  // reads, MFMAs, LDS writes of step s+1); the groups below interleave the
  // non-MFMA stream into the 64-cycle MFMA gaps: each MFMA is followed by one
  // LDS op, every other one by one global load, plus a few VALU.
  auto interleave = [&]() __attribute__((always_inline)) {
    constexpr int NM = RK * RN * (BMR / 2);        // MFMAs per step
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (RK + RN), 0);   // first fragments
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
      __builtin_amdgcn_sched_group_barrier(0x080, 1, 0);              // DS read / write
      if (i % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // global load
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);              // VALU
    }
  };
  // prologue: step 0 -> LDS[0]; step 1 in flight in st1
  if (nsteps > 0) {
    load_step(st0, mbeg);
    store_step(st0, 0);
  }
  if (nsteps > 1) load_step(st1, mbeg + BMR);
  __syncthreads();
  int s = 0;
  for (; s + 1 < nsteps; s += 2) {
    // unconditional loads / stores keep each step ONE scheduling region: past
    // the end the loads are masked to zero (mv) and the stores land in a
    // buffer no later step reads
    load_step(st0, mbeg + (s + 2) * BMR);
    compute(0);
    store_step(st1, 1);
    interleave();
    __syncthreads();
    load_step(st1, mbeg + (s + 3) * BMR);
    compute(1);
    store_step(st0, 0);
    interleave();
    __syncthreads();
  }
  if (s < nsteps) compute(0);   // odd step count: the last step sits in LDS[0]
  // acc[i][j][r]: row k = 32i + (r&3) + 8(r>>2) + 4*lk, col n = 32j + lc
  float* out = a.slab + (long long)split * a.Kp * a.Np;
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = k0 + wk * TK + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const int n = n0 + wnn * TN + 32 * j + lc;
        out[(long long)k * a.Np + n] = acc[i][j][r];
      }
}

// Deterministic split reduction: slab[0][k][n] = sum_s slab[s][k][n] (coalesced).
// In place: row g*gs of each group of gs consecutive split rows gets the group's
// sum (blockIdx.y = group; rows added in order); with gs = splits, row 0 gets
// the total. Two passes (groups, then the group rows at stride gs) keep the
// order fixed and give the few-output / many-split slabs enough workgroups.
__global__ void slab_reduce_kernel(float* slab, int splits, long long per, int gs) {
  const int g0 = blockIdx.y * gs, g1 = min(splits, g0 + gs);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < per;
       i += (long long)gridDim.x * blockDim.x) {
    float s = slab[(long long)g0 * per + i];
    for (int sp = g0 + 1; sp < g1; ++sp) s += slab[(long long)sp * per + i];
    slab[(long long)g0 * per + i] = s;
  }
}
__global__ void slab_gather_kernel(float* slab, int splits, long long per, int gs) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < per;
       i += (long long)gridDim.x * blockDim.x) {
    float s = slab[i];
    for (int sp = gs; sp < splits; sp += gs) s += slab[(long long)sp * per + i];
    slab[i] = s;
  }
}

// ---------------------------------------------------------------------------
// Weight packing / unpacking (the complex block weight, complex_nn.py:52-65)
// ---------------------------------------------------------------------------
// The real-equivalent kernel K(ci, co, i, j) of a complex layer, in terms of
// the (input block, output block) of the channel-stacked tensors:
//   (re, re) -> Wr, (re, im) -> Wi, (im, re) -> -Wi, (im, im) -> Wr.
// Wr/Wi memory layout: conv [Co/2, Ci/2, kh, kw]; convT [Ci/2, Co/2, kh, kw].
struct WeightView {
  const float* wr;
  const float* wi;
  int Ci, Co, kh, kw;
  int transposed, complex_w;
  int sd;          // SE_DTYPE_* of wr / wi
};

__device__ __forceinline__ float kernel_value(const WeightView& w, int ci, int co, int i, int j) {
  if (!w.complex_w) {
    const long long idx = w.transposed ? (((long long)ci * w.Co + co) * w.kh + i) * w.kw + j
                                       : (((long long)co * w.Ci + ci) * w.kh + i) * w.kw + j;
    return ld_any(w.wr, idx, w.sd);
  }
  const int hci = w.Ci / 2, hco = w.Co / 2;
  const bool ci_im = ci >= hci, co_im = co >= hco;
  const int a = ci_im ? ci - hci : ci, b = co_im ? co - hco : co;
  const long long idx = w.transposed ? (((long long)a * hco + b) * w.kh + i) * w.kw + j
                                     : (((long long)b * hci + a) * w.kh + i) * w.kw + j;
  if (ci_im == co_im) return ld_any(w.wr, idx, w.sd);
  return co_im ? ld_any(w.wi, idx, w.sd) : -ld_any(w.wi, idx, w.sd);
}

__device__ __forceinline__ int ilv64_host_dev(int c) { return (c & ~63) | ((c & 31) << 1) | ((c >> 5) & 1); }

struct TapList {
  int n;
  int ti[kMaxTaps], tj[kMaxTaps];     // kernel (i, j) of each tap
  int offh[kMaxTaps], offw[kMaxTaps]; // input offsets
};

// Builds Wp[k = t*Cg + c][n] (zero rows/cols up to Kp x ldw) and ktab[k].
// data_grad = 0: gather channel c is ci, output n is co; 1: c is co, n is ci.
__global__ void prep_class_kernel(WeightView w, TapList taps, int Cg, int N, int Kp, int ldw,
                                  int Hi, int Wi, int data_grad, float* Wp, int4* ktab) {
  const int K = taps.n * Cg;
  const long long total = (long long)Kp * ldw;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(idx / ldw), n = (int)(idx % ldw);
    float v = 0.f;
    if (k < K && n < N) {
      const int t = k / Cg, c = k % Cg;
      const int ci = data_grad ? n : c, co = data_grad ? c : n;
      v = kernel_value(w, ci, co, taps.ti[t], taps.tj[t]);
    }
    Wp[ldw >= 64 ? (long long)k * ldw + ilv64_host_dev(n) : idx] = v;
    if (n == 0) {
      int4 e;
      if (k < K) {
        const int t = k / Cg, c = k % Cg;
        e.x = (int)((long long)c * Hi * Wi + (long long)taps.offh[t] * Wi + taps.offw[t]);
        e.y = taps.offh[t];
        e.z = taps.offw[t];
      } else {
        e.x = 0; e.y = kInvalidOff; e.z = 0;
      }
      e.w = 0;
      ktab[k] = e;
    }
  }
}

#include "cconv_x3.hpp"

// bias_full[n] for the fused complex conv: re = br - bi, im = bi + br.
__global__ void prep_bias_kernel(const float* br, const float* bi, int N, int complex_w, float* out, int sd) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  if (!complex_w) { out[n] = ld_any(br, n, sd); return; }
  const int h = N / 2;
  out[n] = n < h ? ld_any(br, n, sd) - ld_any(bi, n, sd) : ld_any(bi, n - h, sd) + ld_any(br, n - h, sd);
}

// Sums the wgrad slabs and scatters the real-equivalent gradient dK back onto
// dWr / dWi: dWr = dK(re,re) + dK(im,im); dWi = dK(re,im) - dK(im,re).
// dWp layout: [k = t*Cg + c][n]; conv: c = ci, n = co; convT: c = co, n = ci.
struct UnpackArgs {
  const float* slab;
  int splits, Kp, Np;
  float* dwr; float* dwi;
  int Ci, Co, kh, kw, transposed, complex_w;
  int Cg;                                  // gather channels of the wgrad pass
  int tap_of[kMaxTaps];                    // (i*kw + j) -> tap index t
  int sd;                                  // SE_DTYPE_* of dwr / dwi
};

__device__ __forceinline__ float dk_sum(const UnpackArgs& u, int ci, int co, int t) {
  const int c = u.transposed ? co : ci;
  const int n = u.transposed ? ci : co;
  const long long off = (long long)(t * u.Cg + c) * u.Np + n;
  float s = 0.f;
  for (int sp = 0; sp < u.splits; ++sp) s += u.slab[(long long)sp * u.Kp * u.Np + off];
  return s;
}

__global__ void wgrad_finish_kernel(const UnpackArgs u) {
  const int hci = u.complex_w ? u.Ci / 2 : u.Ci, hco = u.complex_w ? u.Co / 2 : u.Co;
  const long long total = (long long)hci * hco * u.kh * u.kw;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    // idx enumerates the weight tensor in memory order
    const int j = (int)(idx % u.kw);
    const int i = (int)((idx / u.kw) % u.kh);
    const long long ab = idx / ((long long)u.kw * u.kh);
    int a0, b0;   // a0 = first dim, b0 = second dim of the weight tensor
    if (u.transposed) { a0 = (int)(ab / hco); b0 = (int)(ab % hco); }
    else { a0 = (int)(ab / hci); b0 = (int)(ab % hci); }
    const int ci = u.transposed ? a0 : b0, co = u.transposed ? b0 : a0;
    const int t = u.tap_of[i * u.kw + j];
    if (!u.complex_w) {
      st_any(u.dwr, idx, dk_sum(u, ci, co, t), u.sd);
      continue;
    }
    const float rr = dk_sum(u, ci, co, t), ii = dk_sum(u, ci + hci, co + hco, t);
    const float ri = dk_sum(u, ci, co + hco, t), ir = dk_sum(u, ci + hci, co, t);
    st_any(u.dwr, idx, rr + ii, u.sd);
    st_any(u.dwi, idx, ri - ir, u.sd);
  }
}

// Bias grad: db_full[n] = sum over (b, h, w) of dy[b, n, h, w]; then fold. One
// block per real channel, or per complex channel pair (n, n + N/2), written
// directly (no zeroed outputs, no atomics): d(br) = sum(dy_re) + sum(dy_im),
// d(bi) = -sum(dy_re) + sum(dy_im), the values the two-atomic form produced.
template <int SD = 0>
__global__ void bias_grad_kernel(const float* dy, int B, int N, long long HW, int complex_w,
                                 float* dbr, float* dbi) {
  const int n = blockIdx.x;
  __shared__ float red[kThreads / 64];
  float t[2] = {0.f, 0.f};
  for (int q = 0; q < (complex_w ? 2 : 1); ++q) {
    const int ch = n + q * (N / 2);
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      const long long p = ((long long)b * N + ch) * HW;
      for (long long i = threadIdx.x; i < HW; i += kThreads) s += ld_s<SD>(dy, p + i);
    }
    s = se::wave_sum(s);
    __syncthreads();   // red is reused by the second channel
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < kThreads / 64; ++i) t[q] += red[i];
  }
  if (threadIdx.x != 0) return;
  if (!complex_w) { st_s<SD>(dbr, n, t[0]); return; }
  st_s<SD>(dbr, n, t[0] + t[1]);
  st_s<SD>(dbi, n, -t[0] + t[1]);
}

// ---------------------------------------------------------------------------
// Host-side planning
// ---------------------------------------------------------------------------
struct Dim1 {   // one spatial dim of one class
  int p, S, Q, s;
  int ntaps;
  int tap[16], off[16];
};

// strided gather: out q in [0, Lout), in = q*stride + i*dil - pad
static Dim1 strided_dim(int Lout, int k, int stride, int pad, int dil) {
  Dim1 d{};
  d.p = 0; d.S = 1; d.Q = Lout; d.s = stride;
  d.ntaps = k;
  for (int i = 0; i < k; ++i) { d.tap[i] = i; d.off[i] = i * dil - pad; }
  return d;
}

// phase-class gather for class p of a stride-`stride` scatter:
// out o = p + stride*q ; in = q + (p + pad - i*dil)/stride for matching taps
static Dim1 phase_dim(int Lout, int k, int stride, int pad, int dil, int p) {
  Dim1 d{};
  d.p = p; d.S = stride; d.s = 1;
  d.Q = Lout > p ? (Lout - p + stride - 1) / stride : 0;
  d.ntaps = 0;
  for (int i = 0; i < k; ++i) {
    const int num = p + pad - i * dil;
    const int r = ((num % stride) + stride) % stride;
    if (r == 0) { d.tap[d.ntaps] = i; d.off[d.ntaps] = num / stride; ++d.ntaps; }
  }
  return d;
}

struct ClassPlan {
  Dim1 h, w;
  TapList taps;
  int K, Kp;
};

static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

static void finish_plan(ClassPlan& c, int Cg, int kstep = kBK) {
  c.taps.n = c.h.ntaps * c.w.ntaps;
  int t = 0;
  for (int a = 0; a < c.h.ntaps; ++a)
    for (int b = 0; b < c.w.ntaps; ++b, ++t) {
      c.taps.ti[t] = c.h.tap[a]; c.taps.tj[t] = c.w.tap[b];
      c.taps.offh[t] = c.h.off[a]; c.taps.offw[t] = c.w.off[b];
    }
  c.K = c.taps.n * Cg;
  c.Kp = round_up(std::max(c.K, 1), kstep);
}

enum Pass { kFwd = 0, kData = 1 };

struct ConvGeom {
  int B, Ci, Hi, Wi, Co, Ho, Wo;
  int kh, kw, sh, sw, ph, pw, dh, dw, oph, opw, transposed, complex_w;
  int phe, pwe;   // end (bottom / right) padding; ph / pw are the begin offsets
  int math;       // SE_MATH_*
  const float* x_amax;    // SE_MATH_F16X3 scale sources from the caller (or nullptr)
  const float* dy_amax;
  const float* w_amax;    // bound of max |w| from the caller (or nullptr)
  int sd;         // se_conv2d_desc.dtype (SE_DTYPE_*)
  int jcat;       // se_conv2d_desc.join_cat
  const void* data_w;   // se_conv2d_desc.data_weights (data-grad weight image, or nullptr)
};

static int geom_of(const se_conv2d_desc* d, ConvGeom& g) {
  if (!d) return SE_E_ARG;
  g.B = d->batch; g.Ci = d->in_channels; g.Hi = d->in_h; g.Wi = d->in_w; g.Co = d->out_channels;
  g.kh = d->kernel_h; g.kw = d->kernel_w; g.sh = d->stride_h; g.sw = d->stride_w;
  g.ph = d->pad_h; g.pw = d->pad_w; g.dh = d->dil_h; g.dw = d->dil_w;
  g.oph = d->out_pad_h; g.opw = d->out_pad_w; g.transposed = d->transposed; g.complex_w = d->complex_weights;
  g.phe = d->pad_h_end < 0 ? g.ph : d->pad_h_end;
  g.pwe = d->pad_w_end < 0 ? g.pw : d->pad_w_end;
  g.math = d->math;
  g.x_amax = d->x_amax;
  g.dy_amax = d->dy_amax;
  g.w_amax = d->w_amax;
  g.sd = d->dtype;
  g.jcat = d->join_cat;
  g.data_w = d->data_weights;
  if (g.jcat != 0 && g.jcat != 1) return SE_E_ARG;
  if (g.math < SE_MATH_F32 || g.math > SE_MATH_F16) return SE_E_ARG;
  if (g.sd < SE_DTYPE_F32 || g.sd > SE_DTYPE_F16) return SE_E_ARG;
  // 16-bit storage runs the one-term MFMA of its own format (operands exact)
  if (g.sd == SE_DTYPE_BF16 && g.math != SE_MATH_BF16) return SE_E_UNSUPPORTED;
  if (g.sd == SE_DTYPE_F16 && g.math != SE_MATH_F16) return SE_E_UNSUPPORTED;
  if (g.B <= 0 || g.Ci <= 0 || g.Co <= 0 || g.Hi <= 0 || g.Wi <= 0 || g.kh <= 0 || g.kw <= 0 ||
      g.sh <= 0 || g.sw <= 0 || g.dh <= 0 || g.dw <= 0 || g.ph < 0 || g.pw < 0)
    return SE_E_ARG;
  if (g.kh > 16 || g.kw > 16 || g.kh * g.kw > kMaxTaps) return SE_E_UNSUPPORTED;
  if (g.complex_w && ((g.Ci & 1) || (g.Co & 1))) return SE_E_SHAPE;
  if (g.transposed) {
    g.Ho = (g.Hi - 1) * g.sh - (g.ph + g.phe) + g.dh * (g.kh - 1) + g.oph + 1;
    g.Wo = (g.Wi - 1) * g.sw - (g.pw + g.pwe) + g.dw * (g.kw - 1) + g.opw + 1;
  } else {
    g.Ho = (g.Hi + g.ph + g.phe - g.dh * (g.kh - 1) - 1) / g.sh + 1;
    g.Wo = (g.Wi + g.pw + g.pwe - g.dw * (g.kw - 1) - 1) / g.sw + 1;
  }
  if (g.Ho <= 0 || g.Wo <= 0) return SE_E_SHAPE;
  return SE_OK;
}

// One-term bf16 (SE_MATH_BF16, the low-precision configs' arithmetic) runs the
// 128-column MFMA tiles down to N = 17: even with 2-4x zero columns a bf16 MFMA tile
// beats the fp32-MFMA tiles (1/16 of the bf16 rate) that the fp32-class modes keep
// for N <= 64 (DCCRN / DCUNet's 32- and 64-channel layers).
static inline bool bf16_tiles(int N, int math) { return (math == SE_MATH_BF16 || math == SE_MATH_F16) && N > 16; }

// Classes of a gather pass. kFwd: conv -> strided, convT -> phase.
// kData: conv -> phase (scatter back), convT -> strided.
static std::vector<ClassPlan> plan_pass(const ConvGeom& g, Pass pass) {
  std::vector<ClassPlan> out;
  const bool phase = (pass == kFwd) ? g.transposed : !g.transposed;
  const int Lh = (pass == kFwd) ? g.Ho : g.Hi, Lw = (pass == kFwd) ? g.Wo : g.Wi;
  const int Cg = (pass == kFwd) ? g.Ci : g.Co;
  // the one-term MFMA tiles stage 64 k per round (gather_x3_kernel<., 1>)
  const int kstep = bf16_tiles((pass == kFwd) ? g.Co : g.Ci, g.math) ? kX3OneTermHalves * kBK : kBK;
  if (!phase) {
    ClassPlan c{};
    c.h = strided_dim(Lh, g.kh, g.sh, g.ph, g.dh);
    c.w = strided_dim(Lw, g.kw, g.sw, g.pw, g.dw);
    finish_plan(c, Cg, kstep);
    out.push_back(c);
    return out;
  }
  for (int p = 0; p < g.sh; ++p)
    for (int q = 0; q < g.sw; ++q) {
      ClassPlan c{};
      c.h = phase_dim(Lh, g.kh, g.sh, g.ph, g.dh, p);
      c.w = phase_dim(Lw, g.kw, g.sw, g.pw, g.dw, q);
      if (c.h.Q == 0 || c.w.Q == 0) continue;
      finish_plan(c, Cg, kstep);
      out.push_back(c);
    }
  return out;
}


static inline int ldw_for(int N, int math = SE_MATH_F32) {
  if (N <= 16) return N <= 4 ? 4 : (N <= 8 ? 8 : 16);  // = the small-N kernel's NOUT
  if (bf16_tiles(N, math)) return round_up(N, 128);
  return round_up(N, N <= 64 ? 64 : 128);
}

// bytes per (k, n) weight element in the workspace: fp32 (4), split bf16 hi/lo
// (4) or the three-way split (6)
constexpr size_t kWpBytesPerElem = 6;

// Channel groups of the chunked stencil (gather_stencil_ch_kernel) for a class of
// B x Qh x Qw outputs over Cg channels: enough workgroups to fill the chip (a B = 16
// DCUNet final layer has ~600 tiles), each group >= 4 chunks of kScC channels.
static int stencil_ch_groups(int B, int Qh, int Qw, int Cg) {
  const long long tiles = (long long)se::ceil_div(Qw, kStW) * se::ceil_div(Qh, kScRows) * B;
  int g = (int)std::max<long long>(1, std::min<long long>(8, 2048 / std::max<long long>(tiles, 1)));
  g = std::min(g, std::max(1, Cg / (4 * kScC)));
  const int cpg = round_up(se::ceil_div(Cg, g), kScC);
  return se::ceil_div(Cg, cpg);
}

static size_t gather_ws_bytes(const std::vector<ClassPlan>& cls, int N, int math = SE_MATH_F32, int B = 0,
                              int Cg = 0) {
  size_t bytes = 0;
  (void)math;   // sized for the wider of the fp32 and bf16 tilings (and the one-term 64-k
                // rounding of Kp): a conv's passes may differ in math
  const int ldw = std::max(ldw_for(N, SE_MATH_F32), ldw_for(N, SE_MATH_BF16));
  size_t part = 0;
  for (const auto& c : cls) {
    bytes += (size_t)round_up(c.Kp, 2 * kBK) * ldw * kWpBytesPerElem;
    bytes += (size_t)round_up(c.Kp, 2 * kBK) * sizeof(int4);
    if (N <= 4 && Cg > 4 && B > 0) {   // the chunked stencil's channel-group partials
      const int gr = stencil_ch_groups(B, c.h.Q, c.w.Q, Cg);
      if (gr > 1) part = std::max(part, (size_t)gr * B * N * c.h.Q * c.w.Q * sizeof(float) + 256);
    }
  }
  bytes += (size_t)round_up(N, 128) * sizeof(float);  // bias_full
  return bytes + part + kZeroBytes + kAmaxBytes + 512;
}

constexpr int kSmallWgradN = 8;   // N at or below: wgrad_smalln_kernel

// wgrad plan: G is gathered (strided) over the grid of D.
struct WgradPlan {
  ClassPlan c;        // strided class over D's grid
  int Cg, N, Qh, Qw;  // gather channels, D channels, D grid
  int Hi, Wi;         // G spatial dims
  int M, splits, m_per_split, Np;
};

static WgradPlan plan_wgrad(const ConvGeom& g) {
  WgradPlan w{};
  if (!g.transposed) {   // G = x strided over y's grid, D = dy
    w.c.h = strided_dim(g.Ho, g.kh, g.sh, g.ph, g.dh);
    w.c.w = strided_dim(g.Wo, g.kw, g.sw, g.pw, g.dw);
    w.Cg = g.Ci; w.N = g.Co; w.Qh = g.Ho; w.Qw = g.Wo; w.Hi = g.Hi; w.Wi = g.Wi;
  } else {               // G = dy strided over x's grid, D = x
    w.c.h = strided_dim(g.Hi, g.kh, g.sh, g.ph, g.dh);
    w.c.w = strided_dim(g.Wi, g.kw, g.sw, g.pw, g.dw);
    w.Cg = g.Co; w.N = g.Ci; w.Qh = g.Hi; w.Qw = g.Wi; w.Hi = g.Ho; w.Wi = g.Wo;
  }
  finish_plan(w.c, w.Cg);
  w.c.Kp = round_up(std::max(w.c.K, 1), 128);
  w.M = g.B * w.Qh * w.Qw;
  if (w.N <= kSmallWgradN) {      // direct kernel: Kp/16 row groups x splits
    w.Np = w.N <= 4 ? 4 : 8;
    const int groups = w.c.Kp / 16;
    int splits = std::max(1, 4096 / groups);
    splits = std::min(splits, std::max(1, w.M / 1024));
    w.m_per_split = (w.M + splits - 1) / splits;
    w.splits = (w.M + w.m_per_split - 1) / w.m_per_split;
    return w;
  }
  // one-term SE_MATH_BF16 / SE_MATH_F16 with N % 16 == 0: the 128-column tiles (see bf16_tiles)
  const bool n32 = w.N <= 32 && !((g.math == SE_MATH_BF16 || g.math == SE_MATH_F16) && w.N % 16 == 0);
  w.Np = round_up(w.N, n32 ? 32 : 128);
  const int tiles = (w.c.Kp / 128) * (w.Np / (n32 ? 32 : 128));
  int splits = std::max(1, 1024 / std::max(tiles, 1));
  // At most kWgradMps positions per m-split: the (k, n) tiles of one split run on
  // one XCD and re-read G and D through its L2; short splits keep them close
  // enough together for those re-reads to hit (dec5 weight-grad FETCH 40-48 ->
  // 29-32 GB, 14.3 -> 12.4 ms; FRCRN step 574 -> 588 utt/s, same box; 2048 and
  // 1024 measured slower).
#ifndef SE_WGRAD_MPS
#define SE_WGRAD_MPS 4096
#endif
  constexpr int kWgradMps = SE_WGRAD_MPS;
  splits = std::max(splits, (w.M + kWgradMps - 1) / kWgradMps);
  const int max_by_m = std::max(1, w.M / 512);
  splits = std::min(splits, max_by_m);
  // keep the slab <= 1 GB
  const size_t per = (size_t)w.c.Kp * w.Np * sizeof(float);
  const size_t cap = 1024ull << 20;
  splits = (int)std::min<size_t>(splits, std::max<size_t>(1, cap / per));
  w.m_per_split = round_up((w.M + splits - 1) / splits, 64);
  w.splits = (w.M + w.m_per_split - 1) / w.m_per_split;
  return w;
}

static size_t wgrad_ws_bytes(const WgradPlan& w) {
  return (size_t)w.splits * w.c.Kp * w.Np * sizeof(float) + (size_t)w.c.Kp * sizeof(int4) +
         kZeroBytes + kAmaxBytes + 512;
}

// SE_MATH_F16X3 scale sources: max |.| of each listed tensor into one slot
// (zeroed with the workspace's zero page). A caller-supplied bound skips the pass.
static void launch_amax(const float* x, long long n, float* slot, hipStream_t st) {
  if (n <= 0) return;
  const long long blocks = std::min<long long>(std::max<long long>((n / 4 + 255) / 256, 1), 2048);
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, (unsigned*)slot);
}

static inline char* align256(char* p) { return (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255); }

// Decoder skip join folded into a gather pass (se_conv2d_*_joined): X of the
// pass is s, x2 is x on its own (h2, w2) grid (gather side); or Y of the pass
// gets the s chunks and y2 the x chunks on (yh2, yw2) (output side).
struct JoinIO {
  const float* x2; int jh, h2, w2;
  int cat;          // se_conv2d_desc.join_cat
  float* y2; int yjh, yh2, yw2;
  const float* s;   // weight-grad: the skip (D of a transposed conv)
};

// SEHIP_STENCIL=0 (tests): the small-N stride-1 convs on gather_smalln_kernel
// instead of the bit-identical LDS stencil
static bool env_flag_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}
static bool env_flag_on(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '1';
}
// The weight image of a gather pass: per stride-phase class the GEMM weight
// tiles Wp (Kp x ldw, in the layout of the kernel the pass runs) and the tap
// table ktab, laid out 256-byte aligned from base. Built by the pass itself in
// its workspace, or ahead of it (data-grad pass: se_conv2d_prep_data_weights).
struct ClassImage {
  float* Wp;
  int4* ktab;
};

static size_t class_images_bytes(const std::vector<ClassPlan>& cls, int ldw) {
  size_t b = 256;
  for (const auto& c : cls)
    b += round_up((long long)c.Kp * ldw * kWpBytesPerElem, 256) + round_up((long long)c.Kp * sizeof(int4), 256);
  return b;
}

// split kernels: channel-block-major K order where Cg allows (split_k)
static int korder_blk(int Cg) { return Cg % 32 == 0 ? 32 : 0; }

static void class_images(const ConvGeom& g, Pass pass, const std::vector<ClassPlan>& cls, int ldw,
                         const WeightView& wv, const float* wamax, char* base, bool build, hipStream_t st,
                         std::vector<ClassImage>& out) {
  const int N = (pass == kFwd) ? g.Co : g.Ci;
  const int Cg = (pass == kFwd) ? g.Ci : g.Co;
  const int Hi = (pass == kFwd) ? g.Hi : g.Ho, Wi = (pass == kFwd) ? g.Wi : g.Wo;
  const bool bf1 = g.math == SE_MATH_BF16 && bf16_tiles(N, g.math);
  const bool h1 = g.math == SE_MATH_F16 && bf16_tiles(N, g.math);
  const bool f16 = g.math == SE_MATH_F16X3 && N > 64;
  const bool x3 = (g.math == SE_MATH_BF16X3 && N > 64) || bf1 || h1 || f16;
  const bool x6 = g.math == SE_MATH_BF16X6 && N > 64;
  const int kblk = korder_blk(Cg);
  const int dg = pass == kData ? 1 : 0;
  char* p = align256(base);
  out.clear();
  for (const auto& c : cls) {
    ClassImage im;
    im.Wp = (float*)p;
    p = align256(p + (size_t)c.Kp * ldw * kWpBytesPerElem);
    im.ktab = (int4*)p;
    p = align256(p + (size_t)c.Kp * sizeof(int4));
    out.push_back(im);
    if (!build) continue;
    const long long tot = (long long)c.Kp * ldw;
    const dim3 grid((unsigned)std::min<long long>((tot + 255) / 256, 4096));
    if (x6)
      hipLaunchKernelGGL(prep_class_x6_kernel, grid, dim3(256), 0, st, wv, c.taps, Cg, N, c.Kp, ldw / 128, Hi,
                         Wi, dg, kblk, (unsigned short*)im.Wp, im.ktab);
    else if (f16 || h1)   // h1: fp16 planes, unscaled (no weight bound)
      hipLaunchKernelGGL(prep_class_x3_kernel<true>, grid, dim3(256), 0, st, wv, c.taps, Cg, N, c.Kp, ldw / 128,
                         Hi, Wi, dg, kblk, (unsigned short*)im.Wp, im.ktab, f16 ? wamax : nullptr);
    else if (x3)
      hipLaunchKernelGGL(prep_class_x3_kernel<false>, grid, dim3(256), 0, st, wv, c.taps, Cg, N, c.Kp, ldw / 128,
                         Hi, Wi, dg, kblk, (unsigned short*)im.Wp, im.ktab, (const float*)nullptr);
    else
      hipLaunchKernelGGL(prep_class_kernel, grid, dim3(256), 0, st, wv, c.taps, Cg, N, c.Kp, ldw, Hi, Wi, dg,
                         im.Wp, im.ktab);
  }
}

static int launch_gather(const ConvGeom& g, Pass pass, const float* X, const float* wr,
                         const float* wi, const float* bias_br, const float* bias_bi, float* Y,
                         void* ws, size_t ws_bytes, hipStream_t st, const JoinIO* jn = nullptr) {
  auto cls = plan_pass(g, pass);
  const int N = (pass == kFwd) ? g.Co : g.Ci;
  const int Cg = (pass == kFwd) ? g.Ci : g.Co;
  const int Hi = (pass == kFwd) ? g.Hi : g.Ho, Wi = (pass == kFwd) ? g.Wi : g.Wo;
  const int Ho = (pass == kFwd) ? g.Ho : g.Hi, Wo = (pass == kFwd) ? g.Wo : g.Wi;
  if (ws_bytes < gather_ws_bytes(cls, N, g.math, g.B, Cg)) return SE_E_WORKSPACE;
  // a prepared split-fp16 image carries the caller's weight bound, which the GEMM unscales by
  if (pass == kData && g.data_w && g.math == SE_MATH_F16X3 && N > 64 && !g.w_amax) return SE_E_ARG;
  const int ldw = ldw_for(N, g.math);
  WeightView wv{wr, wi, g.Ci, g.Co, g.kh, g.kw, g.transposed, g.complex_w, g.sd};
  // 16-bit storage joins on the one-term tiles of its format only (the split forms read fp32)
  if (g.sd != SE_DTYPE_F32 && jn && !(g.math == SE_MATH_BF16 || g.math == SE_MATH_F16)) return SE_E_UNSUPPORTED;

  char* p = align256((char*)ws);
  const float* zero = zero_page();
  if (!zero) return SE_E_LAUNCH;
  float* amax_slot = (float*)(p + kZeroBytes);   // [0] weights, [1] gathered tensor
  {   // the slots are atomicMax targets of launch_amax: zeroed only if a pass fills one
    const float* aa = pass == kFwd ? g.x_amax : g.dy_amax;
    if (g.math == SE_MATH_F16X3 && N > 64 && (!g.w_amax || !aa))
      (void)hipMemsetAsync(amax_slot, 0, kAmaxBytes, st);
  }
  p = align256(p + kZeroBytes + kAmaxBytes);
  float* bias_full = nullptr;
  if (pass == kFwd && bias_br) {
    bias_full = (float*)p;
    p = align256(p + round_up(N, 128) * sizeof(float));
    hipLaunchKernelGGL(prep_bias_kernel, dim3(se::ceil_div(N, 256)), dim3(256), 0, st,
                       bias_br, bias_bi, N, g.complex_w, bias_full, g.sd);
  }
  // split-bf16 / bf16 / split-fp16 GEMM for the 128-column tiles (N > 64); other
  // shapes stay fp32
  const bool bf1 = g.math == SE_MATH_BF16 && bf16_tiles(N, g.math);   // one term: hi*hi (bf16)
  const bool h1 = g.math == SE_MATH_F16 && bf16_tiles(N, g.math);     // one term, fp16, unscaled
  const bool f16 = g.math == SE_MATH_F16X3 && N > 64;            // scaled split-fp16
  const bool x3 = (g.math == SE_MATH_BF16X3 && N > 64) || bf1 || h1 || f16;   // prep / tiles shared
  const bool x6 = g.math == SE_MATH_BF16X6 && N > 64;
  const float* amax_a = pass == kFwd ? g.x_amax : g.dy_amax;
  const float* wamax = g.w_amax ? g.w_amax : amax_slot;   // bound of max |w|
  if (f16) {
    const long long nw = (long long)(g.complex_w ? g.Ci / 2 : g.Ci) * (g.complex_w ? g.Co / 2 : g.Co) * g.kh * g.kw;
    if (!g.w_amax) {
      launch_amax(wr, nw, amax_slot, st);
      if (g.complex_w) launch_amax(wi, nw, amax_slot, st);
    }
    if (!amax_a) {
      launch_amax(X, (long long)g.B * (jn && jn->x2 ? 2 * jn->jh : Cg) * Hi * Wi, amax_slot + 1, st);
      if (jn && jn->x2) launch_amax(jn->x2, (long long)g.B * 2 * jn->jh * jn->h2 * jn->w2, amax_slot + 1, st);
      amax_a = amax_slot + 1;
    }
  }
  const bool join_in = jn && jn->x2, join_out = jn && jn->y2;
  const int cpb = join_in ? 2 * jn->jh : Cg;        // channels per batch item of X
  // TU needs whole K-steps inside one tap and 32-bit buffer offsets over the
  // batch items one M-tile can span (for both sources of a joined gather)
  auto tu_of = [&](const ClassPlan& c) {
    const long long qhw = (long long)c.h.Q * c.w.Q;
    const int bm = ldw == 64 ? 256 : 128;
    const long long span = (bm + qhw - 1) / qhw + 1;
    bool ok = (Cg % kBK == 0) && span * cpb * (long long)Hi * Wi * 4 < (1ll << 31) &&
              (long long)c.Kp * ldw * 4 < (1ll << 31);
    if (join_in) ok = ok && span * cpb * (long long)jn->h2 * jn->w2 * 4 < (1ll << 31);
    return ok;
  };
  // the chunked stencil's shape rules (many-channel stride-1 classes with N <= 4, e.g.
  // DCUNet's final convT), shared by the dispatch below and the joined check
  auto stc_ok = [&](const ClassPlan& c, int& hmin, int& wmin) {
    const int nth = c.h.ntaps, ntw = c.w.ntaps;
    bool hdesc = nth >= 1 && nth <= 4 && ntw >= 1 && c.taps.n <= kMaxTaps;
    for (int t = 0; hdesc && t < c.taps.n; ++t)
      hdesc = c.taps.offh[t] == c.h.off[0] - t / ntw && c.taps.offw[t] == c.w.off[t % ntw];
    int wmax = c.w.off[0];
    wmin = c.w.off[0];
    for (int q = 1; q < ntw; ++q) { wmin = std::min(wmin, c.w.off[q]); wmax = std::max(wmax, c.w.off[q]); }
    hmin = c.h.off[0] - (nth - 1);   // the window's first input row offset
    const long long es = g.sd == SE_DTYPE_F32 ? 4 : 2;
    bool ok = ldw <= 4 && Cg > 4 && c.h.s == 1 && c.w.s == 1 && hdesc && (long long)Cg * Hi * Wi * es < (1ll << 31) &&
              wmax - wmin <= kScPitch - kStW && !env_flag_off("SEHIP_STENCIL");
    // joined: gather side, chunk-aligned sources (either join order)
    if (jn) ok = ok && join_in && !join_out && jn->jh % kScC == 0;
    return ok;
  };
  if (jn) {   // the joined forms exist on the split-bf16 / bf16 tap-uniform kernels and the chunked stencil
    const bool stc = N <= 4 && std::all_of(cls.begin(), cls.end(), [&](const ClassPlan& c) {
      int hm, wm;
      return stc_ok(c, hm, wm);
    });
    if (!stc) {
      if (!(x3 || x6) || (join_out && x6)) return SE_E_UNSUPPORTED;
      for (const auto& c : cls)
        if (!tu_of(c)) return SE_E_UNSUPPORTED;
    }
  }
  // the weight images: prepared by the caller (data-grad pass, desc.data_weights)
  // or built here in ws
  const bool have_img = pass == kData && g.data_w;
  std::vector<ClassImage> img;
  class_images(g, pass, cls, ldw, wv, wamax, have_img ? (char*)g.data_w : p, !have_img, st, img);
  for (size_t ic = 0; ic < cls.size(); ++ic) {
    const ClassPlan& c = cls[ic];
    GatherArgs a{};
    a.X = X; a.ktab = img[ic].ktab; a.Wp = img[ic].Wp; a.bias = bias_full; a.zero = zero; a.Y = Y;
    a.amax_a = amax_a; a.amax_w = wamax;
    a.Cg = Cg; a.Hi = Hi; a.Wi = Wi; a.N = N; a.Ho = Ho; a.Wo = Wo;
    a.ph = c.h.p; a.pw = c.w.p; a.Sh = c.h.S; a.Sw = c.w.S; a.Qh = c.h.Q; a.Qw = c.w.Q;
    a.sh = c.h.s; a.sw = c.w.s; a.Kp = c.Kp; a.ldw = ldw;
    if (jn) {
      a.X2 = jn->x2; a.jh = jn->jh; a.H2 = jn->h2; a.W2 = jn->w2; a.jcat = jn->cat;
      a.Y2 = jn->y2; a.yjh = jn->yjh; a.YH2 = jn->yh2; a.YW2 = jn->yw2;
    }
    const long long M = (long long)g.B * c.h.Q * c.w.Q;
    if (M > INT32_MAX) return SE_E_UNSUPPORTED;
    a.M = (int)M;
    if (N <= 16) {
      // stride-1 single-class small convs (CCBAM's spatial conv and its data-grad): the
      // LDS stencil, bit-identical to gather_smalln_kernel
      int h0 = 0, h1 = 0, w0 = 0, w1 = 0;
      for (int t = 0; t < c.taps.n; ++t) {
        h0 = std::min(h0, c.taps.offh[t]); h1 = std::max(h1, c.taps.offh[t]);
        w0 = std::min(w0, c.taps.offw[t]); w1 = std::max(w1, c.taps.offw[t]);
      }
      const int th = kStRG * kStR + h1 - h0, tw = kStW + w1 - w0;
      const bool stencil = g.sd == SE_DTYPE_F32 && !jn && ldw <= 4 && (Cg == 2 || Cg == 4) &&
                           c.h.s == 1 && c.w.s == 1 && (size_t)Cg * th * tw * sizeof(float) <= 48 * 1024 &&
                           c.taps.n <= kMaxTaps && !env_flag_off("SEHIP_STENCIL");
      if (stencil) {
        a.ntaps = c.taps.n;
        for (int t = 0; t < c.taps.n; ++t) { a.toffh[t] = c.taps.offh[t]; a.toffw[t] = c.taps.offw[t]; }
        const dim3 sgrid(se::ceil_div(c.w.Q, kStW), se::ceil_div(c.h.Q, kStRG * kStR), g.B);
        const size_t shs = (size_t)Cg * th * tw * sizeof(float);
        if (Cg == 4) hipLaunchKernelGGL((gather_stencil_kernel<4, 4>), sgrid, dim3(kThreads), shs, st, a, h0, w0, th, tw);
        else hipLaunchKernelGGL((gather_stencil_kernel<4, 2>), sgrid, dim3(kThreads), shs, st, a, h0, w0, th, tw);
        SE_LAUNCH_CHECK();
        continue;
      }
      // many-channel stride-1 classes (DCUNet's final convT, also over its decoder join): the
      // chunked stencil
      const int nth = c.h.ntaps, ntw = c.w.ntaps;
      int hmin = 0, wmin = 0;
      const bool stencil_ch = stc_ok(c, hmin, wmin);
      if (jn && !stencil_ch) return SE_E_UNSUPPORTED;   // (excluded by the check above)
      if (stencil_ch) {
        a.ntaps = c.taps.n;
        for (int t = 0; t < c.taps.n; ++t) { a.toffh[t] = c.taps.offh[t]; a.toffw[t] = c.taps.offw[t]; }
        // channel groups write partials into the workspace's tail, summed by the reduce pass
        const int ngrp = stencil_ch_groups(g.B, c.h.Q, c.w.Q, Cg);
        const int cpg = round_up(se::ceil_div(Cg, ngrp), kScC);
        float* part = nullptr;
        if (ngrp > 1) {
          const size_t need = (size_t)ngrp * g.B * N * c.h.Q * c.w.Q * sizeof(float);
          part = (float*)align256((char*)ws + ws_bytes - need - 256);
        }
        const dim3 sgrid(se::ceil_div(c.w.Q, kStW), se::ceil_div(c.h.Q, kScRows), g.B * ngrp);
        const size_t shs = (size_t)kScC * (kScRows + nth - 1) * kScPitch * sizeof(float);
#define SE_STC(NO, NTH)                                                                                   \
  do {                                                                                                    \
    if (g.sd == SE_DTYPE_BF16) hipLaunchKernelGGL((gather_stencil_ch_kernel<NO, NTH, 1>), sgrid, dim3(kThreads), shs, st, a, hmin, wmin, ntw, ngrp, cpg, part); \
    else if (g.sd == SE_DTYPE_F16) hipLaunchKernelGGL((gather_stencil_ch_kernel<NO, NTH, 2>), sgrid, dim3(kThreads), shs, st, a, hmin, wmin, ntw, ngrp, cpg, part); \
    else hipLaunchKernelGGL((gather_stencil_ch_kernel<NO, NTH, 0>), sgrid, dim3(kThreads), shs, st, a, hmin, wmin, ntw, ngrp, cpg, part); \
  } while (0)
#define SE_STC_N(NTH) do { if (N <= 2) SE_STC(2, NTH); else SE_STC(4, NTH); } while (0)
        switch (nth) {
          case 1: SE_STC_N(1); break;
          case 2: SE_STC_N(2); break;
          case 3: SE_STC_N(3); break;
          default: SE_STC_N(4); break;
        }
#undef SE_STC_N
#undef SE_STC
        SE_LAUNCH_CHECK();
        if (part) {
          const dim3 rgrid(se::ceil_div((long long)g.B * N * c.h.Q * c.w.Q, kThreads));
          if (g.sd == SE_DTYPE_BF16) hipLaunchKernelGGL(stencil_ch_reduce_kernel<1>, rgrid, dim3(kThreads), 0, st, a, ngrp, part);
          else if (g.sd == SE_DTYPE_F16) hipLaunchKernelGGL(stencil_ch_reduce_kernel<2>, rgrid, dim3(kThreads), 0, st, a, ngrp, part);
          else hipLaunchKernelGGL(stencil_ch_reduce_kernel<0>, rgrid, dim3(kThreads), 0, st, a, ngrp, part);
          SE_LAUNCH_CHECK();
        }
        continue;
      }
      const size_t sh = (size_t)c.Kp * ldw * sizeof(float);
      if (sh > 64 * 1024) return SE_E_UNSUPPORTED;
      dim3 grid(se::ceil_div(M, kThreads));
#define SE_SMALLN(SDV)                                                                                    \
  do {                                                                                                    \
    if (ldw <= 4) hipLaunchKernelGGL((gather_smalln_kernel<4, SDV>), grid, dim3(kThreads), sh, st, a);    \
    else if (ldw <= 8) hipLaunchKernelGGL((gather_smalln_kernel<8, SDV>), grid, dim3(kThreads), sh, st, a); \
    else hipLaunchKernelGGL((gather_smalln_kernel<16, SDV>), grid, dim3(kThreads), sh, st, a);            \
  } while (0)
      if (g.sd == SE_DTYPE_BF16) SE_SMALLN(1);
      else if (g.sd == SE_DTYPE_F16) SE_SMALLN(2);
      else SE_SMALLN(0);
#undef SE_SMALLN
    } else {
      const bool tu = tu_of(c);
      // 256-column workgroups (NW = 2) where the padded column count allows
      const bool wide = ldw % 256 == 0;
      const dim3 grid(se::ceil_div(M, kX3BM), ldw / (wide ? 2 * kX3BN : kX3BN));
      const dim3 blk(wide ? 2 * kThreads : kThreads);
      if (x6) {
        if (wide) {
          if (join_in) hipLaunchKernelGGL((gather_x6_kernel<true, true, 2>), grid, blk, 0, st, a);
          else if (tu) hipLaunchKernelGGL((gather_x6_kernel<true, false, 2>), grid, blk, 0, st, a);
          else hipLaunchKernelGGL((gather_x6_kernel<false, false, 2>), grid, blk, 0, st, a);
        } else {
          if (join_in) hipLaunchKernelGGL((gather_x6_kernel<true, true>), grid, blk, 0, st, a);
          else if (tu) hipLaunchKernelGGL(gather_x6_kernel<true>, grid, blk, 0, st, a);
          else hipLaunchKernelGGL(gather_x6_kernel<false>, grid, blk, 0, st, a);
        }
      } else if (x3) {
        const int terms = bf1 ? 1 : 3;
#define SE_X3_LAUNCH(T, NWV, F)                                                                            \
  do {                                                                                                    \
    if (join_in) hipLaunchKernelGGL((gather_x3_kernel<true, T, 1, NWV, F>), grid, blk, 0, st, a);         \
    else if (join_out) hipLaunchKernelGGL((gather_x3_kernel<true, T, 2, NWV, F>), grid, blk, 0, st, a);   \
    else if (tu) hipLaunchKernelGGL((gather_x3_kernel<true, T, 0, NWV, F>), grid, blk, 0, st, a);         \
    else hipLaunchKernelGGL((gather_x3_kernel<false, T, 0, NWV, F>), grid, blk, 0, st, a);                \
  } while (0)
        if (g.sd != SE_DTYPE_F32) {   // 16-bit storage: the one-term tiles of its format
#define SE_X3_SD(NWV, F, SDV)                                                                              \
  do {                                                                                                    \
    if (join_in) hipLaunchKernelGGL((gather_x3_kernel<true, 1, 1, NWV, F, SDV>), grid, blk, 0, st, a);     \
    else if (join_out) hipLaunchKernelGGL((gather_x3_kernel<true, 1, 2, NWV, F, SDV>), grid, blk, 0, st, a); \
    else if (tu) hipLaunchKernelGGL((gather_x3_kernel<true, 1, 0, NWV, F, SDV>), grid, blk, 0, st, a);     \
    else hipLaunchKernelGGL((gather_x3_kernel<false, 1, 0, NWV, F, SDV>), grid, blk, 0, st, a);            \
  } while (0)
          if (g.sd == SE_DTYPE_BF16 && wide) SE_X3_SD(2, false, 1);
          else if (g.sd == SE_DTYPE_BF16) SE_X3_SD(1, false, 1);
          else if (wide) SE_X3_SD(2, true, 2);
          else SE_X3_SD(1, true, 2);
#undef SE_X3_SD
        } else if (h1 && wide) SE_X3_LAUNCH(1, 2, true);
        else if (h1) SE_X3_LAUNCH(1, 1, true);
        else if (f16 && wide) SE_X3_LAUNCH(3, 2, true);
        else if (f16) SE_X3_LAUNCH(3, 1, true);
        else if (terms == 1 && wide) SE_X3_LAUNCH(1, 2, false);
        else if (terms == 1) SE_X3_LAUNCH(1, 1, false);
        else if (wide) SE_X3_LAUNCH(3, 2, false);
        else SE_X3_LAUNCH(3, 1, false);
#undef SE_X3_LAUNCH
      } else if (ldw == 64) {
        dim3 grid(se::ceil_div(M, 256), 1);
        if (tu) hipLaunchKernelGGL((gather_gemm_kernel<64, 256, 1, 4, true>), grid, dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((gather_gemm_kernel<64, 256, 1, 4, false>), grid, dim3(kThreads), 0, st, a);
      } else {
        dim3 grid(se::ceil_div(M, 128), ldw / 128);
        if (tu) hipLaunchKernelGGL((gather_gemm_kernel<128, 128, 2, 2, true>), grid, dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((gather_gemm_kernel<128, 128, 2, 2, false>), grid, dim3(kThreads), 0, st, a);
      }
    }
    SE_LAUNCH_CHECK();
  }
  return SE_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
// one workgroup: max |.| over wr (and wi), written straight to *out (no zeroed
// slot needed, so no extra launch). 16-B loads, four in flight per thread when
// both tensors are 16-B aligned (a 64x64x5x2 complex weight: 20 per thread).
__device__ __forceinline__ float amax4(f32x4 v) {
  return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}
__global__ void __launch_bounds__(1024) amax_weights_kernel(const float* __restrict__ wr, long long n,
                                                            const float* __restrict__ wi, float* out) {
  float m = 0.f;
  long long i0 = 0;
  if ((((unsigned long long)wr | (unsigned long long)wi) & 15) == 0) {
    const long long n4 = n >> 2;
    const f32x4* r4 = reinterpret_cast<const f32x4*>(wr);
    const f32x4* i4 = reinterpret_cast<const f32x4*>(wi);
    long long i = threadIdx.x;
    for (; i + 3 * 1024 < n4; i += 4 * 1024) {
      f32x4 v[4], u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = r4[i + q * 1024];
      if (wi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) u[q] = i4[i + q * 1024];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) m = fmaxf(m, wi ? fmaxf(amax4(v[q]), amax4(u[q])) : amax4(v[q]));
    }
    for (; i < n4; i += 1024) m = fmaxf(m, wi ? fmaxf(amax4(r4[i]), amax4(i4[i])) : amax4(r4[i]));
    i0 = 4 * n4;
  }
  for (long long i = i0 + threadIdx.x; i < n; i += 1024) {
    m = fmaxf(m, fabsf(wr[i]));
    if (wi) m = fmaxf(m, fabsf(wi[i]));
  }
  m = se::wave_max(m);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) m = fmaxf(m, red[w]);
    *out = m;
  }
}

extern "C" int se_amax_weights(const float* wr, long long n, const float* wi, float* amax, void* stream) {
  if (!wr || !amax || n < 0) return SE_E_ARG;
  hipLaunchKernelGGL(amax_weights_kernel, dim3(1), dim3(1024), 0, se::as_stream(stream), wr, n, wi, amax);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_amax(const float* x, long long n, float* amax, void* stream) {
  if (!x || !amax || n < 0) return SE_E_ARG;
  launch_amax(x, n, amax, se::as_stream(stream));
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_amax_init(const float* x, long long n, float* amax, void* stream) {
  if (!x || !amax || n < 0) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  if (hipMemsetAsync(amax, 0, sizeof(float), st) != hipSuccess) return SE_E_LAUNCH;
  launch_amax(x, n, amax, st);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_conv2d_out_shape(const se_conv2d_desc* d, int* out_h, int* out_w) {
  ConvGeom g;
  const int rc = geom_of(d, g);
  if (rc) return rc;
  if (out_h) *out_h = g.Ho;
  if (out_w) *out_w = g.Wo;
  return SE_OK;
}

extern "C" size_t se_conv2d_workspace_size(const se_conv2d_desc* d) {
  ConvGeom g;
  if (geom_of(d, g)) return 0;
  size_t a = gather_ws_bytes(plan_pass(g, kFwd), g.Co, g.math, g.B, g.Ci);
  size_t b = gather_ws_bytes(plan_pass(g, kData), g.Ci, g.math, g.B, g.Co);
  size_t c = wgrad_ws_bytes(plan_wgrad(g));
  {   // the weight-grad pass may run in another math than the forward (per-pass modes)
    ConvGeom g2 = g;
    g2.math = g.math == SE_MATH_BF16 ? SE_MATH_F32 : SE_MATH_BF16;
    c = std::max(c, wgrad_ws_bytes(plan_wgrad(g2)));
  }
  return std::max(a, std::max(b, c));
}

extern "C" int se_conv2d_fwd(const se_conv2d_desc* d, const float* x, const float* wr,
                             const float* wi, const float* br, const float* bi, float* y,
                             void* ws, size_t ws_bytes, void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if (!x || !wr || !y || !ws || (g.complex_w && !wi) || (g.complex_w && br && !bi)) return SE_E_ARG;
  return launch_gather(g, kFwd, x, wr, wi, br, bi, y, ws, ws_bytes, se::as_stream(stream));
}

extern "C" size_t se_conv2d_data_weights_size(const se_conv2d_desc* d) {
  ConvGeom g;
  if (geom_of(d, g)) return 0;
  return class_images_bytes(plan_pass(g, kData), ldw_for(g.Ci, g.math));
}

extern "C" int se_conv2d_prep_data_weights(const se_conv2d_desc* d, const float* wr, const float* wi,
                                           void* img, size_t img_bytes, void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if (!wr || !img || (g.complex_w && !wi)) return SE_E_ARG;
  if (g.math == SE_MATH_F16X3 && g.Ci > 64 && !g.w_amax) return SE_E_ARG;
  const auto cls = plan_pass(g, kData);
  const int ldw = ldw_for(g.Ci, g.math);
  if (img_bytes < class_images_bytes(cls, ldw)) return SE_E_WORKSPACE;
  const WeightView wv{wr, wi, g.Ci, g.Co, g.kh, g.kw, g.transposed, g.complex_w, g.sd};
  std::vector<ClassImage> out;
  class_images(g, kData, cls, ldw, wv, g.w_amax, (char*)img, true, se::as_stream(stream), out);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_conv2d_bwd_data(const se_conv2d_desc* d, const float* dy, const float* wr,
                                  const float* wi, float* dx, void* ws, size_t ws_bytes,
                                  void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if (!dy || !wr || !dx || !ws || (g.complex_w && !wi)) return SE_E_ARG;
  // the phase classes tile dx completely; positions hit by no tap get 0
  return launch_gather(g, kData, dy, wr, wi, nullptr, nullptr, dx, ws, ws_bytes,
                       se::as_stream(stream));
}

namespace {

// 1-D grid of wgrad_x3_kernel over its tile space (a.vk k-tiles x a.vn n-tiles x
// a.vs m-splits, one workgroup each). nb: 128-row D blocks per workgroup.
dim3 x3_wgrad_grid(WgradArgs& a, const WgradPlan& w, int nb = 1, int kb = 1) {
  a.vk = w.c.Kp / (128 * kb); a.vn = w.Np / (128 * nb); a.vs = w.splits;
  return dim3((unsigned)(a.vk * a.vn * a.vs));
}

// Weight-grad pass. jn (transposed convs only): the conv's input x is the
// decoder skip join, D = s with D2 = jn->x2 on (h2, w2) (se_conv2d_bwd_weight_joined).
int wgrad_pass(const ConvGeom& g, const float* x, const float* dy, float* dwr, float* dwi,
               float* dbr, float* dbi, void* ws, size_t ws_bytes, hipStream_t st,
               const JoinIO* jn = nullptr) {
  WgradPlan w = plan_wgrad(g);
  if (ws_bytes < wgrad_ws_bytes(w)) return SE_E_WORKSPACE;
  const long long QQw = (long long)w.Qh * w.Qw;
  const long long span_w = (w.m_per_split + QQw - 1) / QQw + 1;
  // the split-bf16 / bf16 tile reads D rows in blocks of 16 (N % 16 == 0)
  const bool split_ok = (g.math == SE_MATH_BF16X3 || g.math == SE_MATH_BF16 || g.math == SE_MATH_F16X3 ||
                         g.math == SE_MATH_F16) && w.N % 16 == 0;
  // 16-bit storage: the one-term split tiles only (the fp32 kernels read fp32)
  if (g.sd != SE_DTYPE_F32 && (!split_ok || w.N <= kSmallWgradN || w.Np == 32))
    return SE_E_UNSUPPORTED;
  if (jn) {
    // the joined D operand (either gather form of G): 32-bit offsets from the split's
    // first batch item; one-term fp16 on fp32 storage has no joined instantiation
    const int dcpb = 2 * jn->jh;
    const bool dj_ok = g.transposed && span_w * dcpb * QQw * 4 < (1ll << 31) &&
                       span_w * dcpb * (long long)jn->h2 * jn->w2 * 4 < (1ll << 31);
    if (!dj_ok || !split_ok || w.N <= 32 || w.N != 4 * jn->jh ||
        (g.math == SE_MATH_F16 && g.sd == SE_DTYPE_F32))
      return SE_E_UNSUPPORTED;
  }
  char* p = align256((char*)ws);
  const float* zero = zero_page();
  if (!zero) return SE_E_LAUNCH;
  float* amax_slot = (float*)(p + kZeroBytes);   // [0] x (joined: x and s), [1] dy
  if (g.math == SE_MATH_F16X3 && (!g.x_amax || !g.dy_amax))   // launch_amax targets below
    (void)hipMemsetAsync(amax_slot, 0, kAmaxBytes, st);
  p = align256(p + kZeroBytes + kAmaxBytes);
  float* slab = (float*)p;
  p = align256(p + (size_t)w.splits * w.c.Kp * w.Np * sizeof(float));
  int4* ktab = (int4*)p;

  // every wgrad_x3_kernel launch below (split or one-term tiles) computes its tap table in
  // the kernel; the fp32 / 32-column / small-N kernels read the prep pass's
  const bool x3_path = split_ok && w.N > kSmallWgradN && w.Np != 32 && w.c.taps.n <= kMaxTaps;
  // ktab only (no weights): reuse prep_class_kernel with ldw = 1 writing into slab[0]
  // would clobber; build it with a one-column pass into a scratch row instead. The
  // split-fp16 weight-grad kernel computes its entries itself (no launch).
  if (!x3_path) {
    WeightView wv{nullptr, nullptr, g.Ci, g.Co, g.kh, g.kw, g.transposed, 0};
    // N = 0 -> every Wp entry is 0 and only ktab matters; Wp scratch = slab start
    hipLaunchKernelGGL(prep_class_kernel, dim3(se::ceil_div(w.c.Kp, 256)), dim3(256), 0, st, wv,
                       w.c.taps, w.Cg, 0, w.c.Kp, 1, w.Hi, w.Wi, 0, slab, ktab);
  }
  WgradArgs a{};
  a.X = g.transposed ? dy : x;
  a.D = g.transposed ? x : dy;
  a.ktab = x3_path ? nullptr : ktab; a.slab = slab; a.zero = zero;
  a.ntaps = w.c.taps.n;
  for (int t = 0; t < w.c.taps.n && t < kMaxTaps; ++t) { a.toffh[t] = w.c.taps.offh[t]; a.toffw[t] = w.c.taps.offw[t]; }
  a.Cg = w.Cg; a.Hi = w.Hi; a.Wi = w.Wi;
  a.N = w.N; a.Qh = w.Qh; a.Qw = w.Qw; a.sh = w.c.h.s; a.sw = w.c.w.s;
  a.Kp = w.c.Kp; a.Np = w.Np; a.M = w.M; a.m_per_split = w.m_per_split;
  if (jn) {
    a.D = jn->s; a.D2 = jn->x2; a.djh = jn->jh; a.DH2 = jn->h2; a.DW2 = jn->w2; a.djcat = jn->cat;
  }
  const bool f16 = split_ok && g.math == SE_MATH_F16X3 && w.N > 32;
  if (f16) {   // scale sources of x (conv input) and dy, unless the caller has them
    const float* xa = g.x_amax;
    const float* da = g.dy_amax;
    if (!xa) {
      if (jn) {
        launch_amax(jn->s, (long long)g.B * 2 * jn->jh * g.Hi * g.Wi, amax_slot, st);
        launch_amax(jn->x2, (long long)g.B * 2 * jn->jh * jn->h2 * jn->w2, amax_slot, st);
      } else {
        launch_amax(x, (long long)g.B * g.Ci * g.Hi * g.Wi, amax_slot, st);
      }
      xa = amax_slot;
    }
    if (!da) {
      launch_amax(dy, (long long)g.B * g.Co * g.Ho * g.Wo, amax_slot + 1, st);
      da = amax_slot + 1;
    }
    a.amax_g = g.transposed ? da : xa;
    a.amax_d = g.transposed ? xa : da;
  }
  const bool tu = (w.Cg % 128 == 0) && span_w * w.Cg * (long long)w.Hi * w.Wi * 4 < (1ll << 31) &&
                  span_w * (long long)w.Np * QQw * 4 < (1ll << 31);
  if (w.N <= kSmallWgradN) {
    dim3 grid(w.c.Kp / 16, w.splits);
    if (w.Np == 4) hipLaunchKernelGGL(wgrad_smalln_kernel<4>, grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL(wgrad_smalln_kernel<8>, grid, dim3(kThreads), 0, st, a);
  } else if (w.Np == 32) {
    dim3 grid(w.c.Kp / 128, 1, w.splits);
    if (tu) hipLaunchKernelGGL((wgrad_gemm_kernel<128, 32, 4, 1, 64, true>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_gemm_kernel<128, 32, 4, 1, 64, false>), grid, dim3(kThreads), 0, st, a);
  } else if (f16 && w.Np % 256 == 0 && tu && w.c.Kp % 256 == 0) {
    // 256 x 256 tiles, 8 waves of 128 x 64: dec5 weight-grad 12.7 -> 10.7 ms, FRCRN step
    // 99.6 -> 96.3 ms (same box), all 167 gradients bit-identical
    const dim3 grid = x3_wgrad_grid(a, w, 2, 2);
    const dim3 blk(2 * kThreads);
    if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, true, true, 2, false, 0, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, false, true, 2, false, 0, 2>), grid, blk, 0, st, a);
  } else if (f16 && w.Np == 128 && tu && !jn && w.c.Kp % 256 == 0 && env_flag_on("SEHIP_WGRAD_K256")) {
    // 256 x 128 tiles, 8 waves of 64 x 64 (the encoder's N = 128): a staged dy row serves two
    // taps' 256 k rows. PMC 3.16 -> 2.39 GB per encoder launch, but 3.62 -> 3.80 ms alone and
    // 10.5 -> 12.0 ms per step (one register staging set at one workgroup per CU): opt-in
    // (profiles/ab/r6_wgrad_256x128_ab.log)
    const dim3 grid = x3_wgrad_grid(a, w, 1, 2);
    hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, false, true, 1, false, 0, 2>), grid, dim3(2 * kThreads), 0, st, a);
  } else if (f16 && w.Np % 256 == 0) {   // 128 x 256 tiles, 8 waves
    const dim3 grid = x3_wgrad_grid(a, w, 2);
    const dim3 blk(2 * kThreads);
    if (jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, true, true, 2>), grid, blk, 0, st, a);
    else if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, true, true, 2>), grid, blk, 0, st, a);
    else if (tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, false, true, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, false, true, 2>), grid, blk, 0, st, a);
  } else if (f16) {
    const dim3 grid = x3_wgrad_grid(a, w);
    const bool kpad = (w.c.taps.n * w.Cg) % 128 != 0;   // e.g. a first conv: K = 10 taps x 2
    if (jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, true, true>), grid, dim3(kThreads), 0, st, a);
    else if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, true, true>), grid, dim3(kThreads), 0, st, a);
    else if (tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, false, true>), grid, dim3(kThreads), 0, st, a);
    else if (kpad) hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, false, true, 1, true>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, false, true>), grid, dim3(kThreads), 0, st, a);
  } else if (split_ok && g.math == SE_MATH_BF16X3) {
    const dim3 grid = x3_wgrad_grid(a, w);
    if (jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 3, true>), grid, dim3(kThreads), 0, st, a);
    else if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 3, true>), grid, dim3(kThreads), 0, st, a);
    else if (tu) hipLaunchKernelGGL(wgrad_x3_kernel<true>, grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL(wgrad_x3_kernel<false>, grid, dim3(kThreads), 0, st, a);
  } else if (split_ok && (g.sd != SE_DTYPE_F32 || g.math == SE_MATH_BF16) && w.Np % 256 == 0 && tu &&
             w.c.Kp % 256 == 0) {
    // one term on 256 x 256 tiles (as the split-fp16 ones above): DCCRN-CL bf16 train step
    // 1276 -> 1321 utt/s (same box, profiles/ab/r5_wgrad_256x256_one_term_configs_ab.log)
    const dim3 grid = x3_wgrad_grid(a, w, 2, 2);
    const dim3 blk(2 * kThreads);
    if (g.sd == SE_DTYPE_BF16 && jn) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true, false, 2, false, 1, 2>), grid, blk, 0, st, a);
    else if (g.sd == SE_DTYPE_BF16) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, false, 2, false, 1, 2>), grid, blk, 0, st, a);
    else if (g.sd == SE_DTYPE_F16 && jn) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true, true, 2, false, 2, 2>), grid, blk, 0, st, a);
    else if (g.sd == SE_DTYPE_F16) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, true, 2, false, 2, 2>), grid, blk, 0, st, a);
    else if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true, false, 2, false, 0, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, false, 2, false, 0, 2>), grid, blk, 0, st, a);
  } else if (split_ok && g.sd != SE_DTYPE_F32) {   // 16-bit storage, one term of its format
    const dim3 grid = x3_wgrad_grid(a, w);
    if (g.sd == SE_DTYPE_BF16 && jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true, false, 1, false, 1>), grid, dim3(kThreads), 0, st, a);
    else if (g.sd == SE_DTYPE_BF16 && jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, true, false, 1, false, 1>), grid, dim3(kThreads), 0, st, a);
    else if (g.sd == SE_DTYPE_F16 && jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true, true, 1, false, 2>), grid, dim3(kThreads), 0, st, a);
    else if (g.sd == SE_DTYPE_F16 && jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, true, true, 1, false, 2>), grid, dim3(kThreads), 0, st, a);
    else if (g.sd == SE_DTYPE_BF16 && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, false, 1, false, 1>), grid, dim3(kThreads), 0, st, a);
    else if (g.sd == SE_DTYPE_BF16) hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, false, false, 1, false, 1>), grid, dim3(kThreads), 0, st, a);
    else if (tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, true, 1, false, 2>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, false, true, 1, false, 2>), grid, dim3(kThreads), 0, st, a);
  } else if (split_ok && g.math == SE_MATH_F16) {   // one-term fp16 on fp32 storage
    const dim3 grid = x3_wgrad_grid(a, w);
    if (tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, false, true>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, false, true>), grid, dim3(kThreads), 0, st, a);
  } else if (split_ok) {   // SE_MATH_BF16
    const dim3 grid = x3_wgrad_grid(a, w);
    if (jn && tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1, true>), grid, dim3(kThreads), 0, st, a);
    else if (jn) hipLaunchKernelGGL((wgrad_x3_kernel<false, 1, true>), grid, dim3(kThreads), 0, st, a);
    else if (tu) hipLaunchKernelGGL((wgrad_x3_kernel<true, 1>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_x3_kernel<false, 1>), grid, dim3(kThreads), 0, st, a);
  } else {
    dim3 grid(w.c.Kp / 128, w.Np / 128, w.splits);
    if (tu) hipLaunchKernelGGL((wgrad_gemm_kernel<128, 128, 2, 2, 32, true>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((wgrad_gemm_kernel<128, 128, 2, 2, 32, false>), grid, dim3(kThreads), 0, st, a);
  }
  SE_LAUNCH_CHECK();

  const long long per = (long long)w.c.Kp * w.Np;
  if (w.splits > 1) {
    const unsigned bx = (unsigned)std::min<long long>((per + 255) / 256, 2048);
    // groups of >= 16 splits until ~2048 workgroups
    int ng = std::max(1, std::min<int>(w.splits / 16, 2048 / (int)bx));
    const int gs = se::ceil_div(w.splits, ng);
    ng = se::ceil_div(w.splits, gs);
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(bx, ng), dim3(256), 0, st, slab, w.splits, per, gs);
    SE_LAUNCH_CHECK();
    if (ng > 1) {
      hipLaunchKernelGGL(slab_gather_kernel, dim3(bx), dim3(256), 0, st, slab, w.splits, per, gs);
      SE_LAUNCH_CHECK();
    }
  }
  UnpackArgs u{};
  u.slab = slab; u.splits = 1; u.Kp = w.c.Kp; u.Np = w.Np;
  u.dwr = dwr; u.dwi = dwi; u.Ci = g.Ci; u.Co = g.Co; u.kh = g.kh; u.kw = g.kw;
  u.transposed = g.transposed; u.complex_w = g.complex_w; u.Cg = w.Cg; u.sd = g.sd;
  for (int t = 0; t < w.c.taps.n; ++t) u.tap_of[w.c.taps.ti[t] * g.kw + w.c.taps.tj[t]] = t;
  const long long nw = (long long)(g.complex_w ? g.Ci / 2 : g.Ci) * (g.complex_w ? g.Co / 2 : g.Co) * g.kh * g.kw;
  hipLaunchKernelGGL(wgrad_finish_kernel, dim3((unsigned)std::min<long long>((nw + 255) / 256, 4096)),
                     dim3(256), 0, st, u);
  SE_LAUNCH_CHECK();

  if (dbr) {
    const int hco = g.complex_w ? g.Co / 2 : g.Co;
    if (g.sd == SE_DTYPE_BF16)
      hipLaunchKernelGGL(bias_grad_kernel<1>, dim3(hco), dim3(kThreads), 0, st, dy, g.B, g.Co,
                         (long long)g.Ho * g.Wo, g.complex_w, dbr, dbi);
    else if (g.sd == SE_DTYPE_F16)
      hipLaunchKernelGGL(bias_grad_kernel<2>, dim3(hco), dim3(kThreads), 0, st, dy, g.B, g.Co,
                         (long long)g.Ho * g.Wo, g.complex_w, dbr, dbi);
    else
      hipLaunchKernelGGL(bias_grad_kernel<0>, dim3(hco), dim3(kThreads), 0, st, dy, g.B, g.Co,
                         (long long)g.Ho * g.Wo, g.complex_w, dbr, dbi);
    SE_LAUNCH_CHECK();
  }
  return SE_OK;
}

// Shape rules of the joined entry points: complex conv over the joined input
// [B, Ci, Hi, Wi] = complex_concat([align(x), s]) with s [B, Ci/2, Hi, Wi] and
// x [B, Ci/2, x_h, x_w], x_h <= Hi (missing rows: F.pad zeros), x_w >= Wi
// (extra columns: x[..., :-1]); chunks of Ci/4 channels, a multiple of 32.
// jh_align: the join blocks' channel alignment the pass's kernels need (32: a GEMM tile's
// 32-row block lies in one chunk; 8: the chunked stencil's channel chunks, the forward of a
// <= 4-output layer such as DCCRN's last decoder convT, jh = 16)
int joined_geom(const ConvGeom& g, int x_h, int x_w, int jh_align = 32) {
  if (!g.complex_w) return SE_E_UNSUPPORTED;
  // complex_concat (FRCRN / DCCRN): x's missing rows read 0, its extra columns are cropped;
  // torch.cat (DCUNet): x is zero-padded to the skip's grid in both dimensions
  if (x_h <= 0 || x_w <= 0 || x_h > g.Hi || (g.jcat ? x_w > g.Wi : x_w < g.Wi)) return SE_E_SHAPE;
  if (g.Ci % 4 || (g.Ci / 4) % jh_align) return SE_E_UNSUPPORTED;
  return SE_OK;
}

}  // namespace

extern "C" int se_conv2d_bwd_weight(const se_conv2d_desc* d, const float* x, const float* dy,
                                    float* dwr, float* dwi, float* dbr, float* dbi, void* ws,
                                    size_t ws_bytes, void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if (!x || !dy || !dwr || !ws || (g.complex_w && !dwi) || (g.complex_w && dbr && !dbi))
    return SE_E_ARG;
  return wgrad_pass(g, x, dy, dwr, dwi, dbr, dbi, ws, ws_bytes, se::as_stream(stream));
}

extern "C" int se_conv2d_fwd_joined(const se_conv2d_desc* d, const float* x, int x_h, int x_w,
                                    const float* s, const float* wr, const float* wi,
                                    const float* br, const float* bi, float* y, void* ws,
                                    size_t ws_bytes, void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if ((rc = joined_geom(g, x_h, x_w, g.Co <= 4 ? 8 : 32))) return rc;
  if (!x || !s || !wr || !wi || !y || !ws || (br && !bi)) return SE_E_ARG;
  JoinIO jn{};
  jn.x2 = x; jn.jh = g.Ci / 4; jn.h2 = x_h; jn.w2 = x_w; jn.cat = g.jcat;
  return launch_gather(g, kFwd, s, wr, wi, br, bi, y, ws, ws_bytes, se::as_stream(stream), &jn);
}

extern "C" int se_conv2d_bwd_data_joined(const se_conv2d_desc* d, const float* dy, const float* wr,
                                         const float* wi, float* gx, int x_h, int x_w, float* gs,
                                         void* ws, size_t ws_bytes, void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if ((rc = joined_geom(g, x_h, x_w))) return rc;
  if (!dy || !wr || !wi || !gx || !gs || !ws) return SE_E_ARG;
  hipStream_t st = se::as_stream(stream);
  JoinIO jn{};
  jn.y2 = gx; jn.yjh = g.Ci / 4; jn.yh2 = x_h; jn.yw2 = x_w; jn.cat = g.jcat;
  if ((rc = launch_gather(g, kData, dy, wr, wi, nullptr, nullptr, gs, ws, ws_bytes, st, &jn))) return rc;
  // x's cropped columns (x[..., :-1]) get a zero gradient
  if (x_w > g.Wi) {
    const size_t rows = (size_t)g.B * (g.Ci / 2) * x_h, es = g.sd == SE_DTYPE_F32 ? 4 : 2;
    if (hipMemset2DAsync((char*)gx + g.Wi * es, (size_t)x_w * es, 0, (size_t)(x_w - g.Wi) * es, rows, st) !=
        hipSuccess)
      return SE_E_LAUNCH;
  }
  return SE_OK;
}

extern "C" int se_conv2d_bwd_weight_joined(const se_conv2d_desc* d, const float* x, int x_h, int x_w,
                                           const float* s, const float* dy, float* dwr, float* dwi,
                                           float* dbr, float* dbi, void* ws, size_t ws_bytes,
                                           void* stream) {
  ConvGeom g;
  int rc = geom_of(d, g);
  if (rc) return rc;
  if ((rc = joined_geom(g, x_h, x_w))) return rc;
  if (!x || !s || !dy || !dwr || !dwi || !ws || (dbr && !dbi)) return SE_E_ARG;
  if (!g.transposed) return SE_E_UNSUPPORTED;   // a plain conv would gather the join as G
  JoinIO jn{};
  jn.s = s; jn.x2 = x; jn.jh = g.Ci / 4; jn.h2 = x_h; jn.w2 = x_w; jn.cat = g.jcat;
  return wgrad_pass(g, s, dy, dwr, dwi, dbr, dbi, ws, ws_bytes, se::as_stream(stream), &jn);
}
