// Plain (batched) GEMMs of the LSTM layers on the scaled split-fp16 MFMA
// ("f16x3", the arithmetic of the conv GEMMs, cconv_x3.hpp): the input
// projection X W_ih^T + b_ih + b_hh, the input gradient dgates W_ih and the
// weight gradients dgates^T X, dgates^T h_prev of torch.nn.LSTM as ComplexLSTM
// runs it (complex_nn.py:115-145); plus the bias gradient as a column sum.
//
// C[b](m, n) = sum_k A(b, m, k) B(b, k, n)   (+ bias0[n] + bias1[n])
//   A(b, m, k) = A[b sa + m lda + k]  (a_mcontig = 0)  or  A[b sa + k lda + m]  (1)
//   B(b, k, n) = B[b sb + n ldb + k]  (b_ncontig = 0)  or  B[b sb + k ldb + n]  (1)
// sum_batches = 1 adds the batch products into one C (dx of a layer whose
// input feeds several LSTMs). A(m, k) is read as 0 where k % kmask_period ==
// kmask_phase: dW_hh = sum_t dgates_t^T h_{t-1} over the flattened (b, t) rows
// without the pairs that straddle two sequences.
//
// Each operand gets a power-of-two scale s = 2^(14 - e) from a bound of its
// max |.| and a hi + lo fp16 split (22 significant bits); a*b ~ hh + hl + lh on
// v_mfma_f32_32x32x16_f16 with fp32 accumulation; the epilogue multiplies by
// 2^(ea + eb - 28) (exact). 128 x 128 tiles of 4 waves (64 x 64 each), 32-deep
// K-steps staged through a double-buffered LDS image in the conv kernels'
// swizzled [plane][row][4 x 16 B] layout. Long reductions (the weight
// gradients: K = B*T rows) are split over K into fp32 slabs, added in split
// order by gemm_reduce_kernel (deterministic).
//
// 16-bit storage (se_gemm_desc.dtype = SE_DTYPE_BF16 / _F16, ABI 10: the
// Linear layers of a model.to(bfloat16) / .half() model, nn.Linear's own
// arithmetic): A, B, C and the biases are read and written in that format,
// the products run on the one-term v_mfma_f32_32x32x16_{bf16,f16} (exact
// products, fp32 accumulation), no scales; C is rounded once. bias_rows = 1
// adds the bias by row m instead of column n (a Linear evaluated as W x^T,
// whose output rows are the features).
#include "common.hpp"

#include <algorithm>

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTop = 14;                 // scaled values stay below 2^14 (fp16 max 65504)
constexpr int kBM = 128, kBN = 128, kBK = 32, kThr = 256;

__device__ __forceinline__ int amax_exp(const float* amax) {   // e with *amax < 2^e
  const unsigned bits = __builtin_bit_cast(unsigned, *amax) & 0x7fffffffu;
  const int e = (int)(bits >> 23) - 126;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}
__device__ __forceinline__ float pow2f(int e) { return __builtin_bit_cast(float, (unsigned)(127 + e) << 23); }

// (x0, x1) * s -> packed fp16 hi pair and lo pair (v_cvt_pk_f16_f32 rounds to nearest even)
__device__ __forceinline__ void split_f16x2(float x0, float x1, float s, unsigned& hi, unsigned& lo) {
  const f32x2 v = (f32x2){x0, x1} * s;
  const f16x2 h = __builtin_convertvector(v, f16x2);
  hi = __builtin_bit_cast(unsigned, h);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(v - __builtin_convertvector(h, f32x2), f16x2));
}

// storage formats: S = float (split-fp16 x3 arithmetic), __bf16 / _Float16 (one term)
template <typename S> constexpr bool is16() { return sizeof(S) == 2; }
template <typename S>
__device__ __forceinline__ f32x16 mfma1(u32x4 a, u32x4 b, f32x16 c) {
  if constexpr (__is_same(S, __bf16))
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

// 16-B chunk c of image row `row` sits at c ^ swz(row): the 32x32x16 fragment
// reads (lane -> row l & 31, chunk 2 ks + (l >> 5)) are conflict-free
__device__ __forceinline__ int swz(int row) { return (row >> 2) & 3; }

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const void* bias0;
  const void* bias1;
  const float* amax_a;
  const float* amax_b;
  float* slab;                 // splits > 1: [nbz][splits][M][N]
  long long sa, sb, sc, sbias;
  int lda, ldb, ldc;
  int M, N, K;
  int nb, sum_b;
  int splits, kps;             // K-steps per split
  int kmask_T, kmask_p;
  int vec_a, vec_b;            // the K-contiguous operand may use 16-B loads
  int bias_rows;               // bias by row m (1) or column n (0)
};

// 16 consecutive k of one row of a K-contiguous operand (row stride ld): 16-B
// loads when the row segment is in range and aligned, else guarded scalars
__device__ __forceinline__ void load_krow(const float* p, bool rok, int kleft, bool vec, float (&v)[16]) {
  if (rok && vec && kleft >= 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 t = reinterpret_cast<const f32x4*>(p)[q];
      v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (rok && j < kleft) ? p[j] : 0.f;
  }
}

// 16 consecutive k (stride ld) of one row of a row-contiguous operand: a wave's
// lanes take 64 consecutive rows, so every load is one 256-B segment
__device__ __forceinline__ void load_kcol(const float* p, long long ld, bool rok, int kleft, float (&v)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = (rok && j < kleft) ? p[(long long)j * ld] : 0.f;
}

// 16-bit storage: the 16 values as the 8 packed pairs the MFMA operand image holds
// (element 2i in the low half of word i), straight from memory; 0 bits are +0
__device__ __forceinline__ void load_krow16(const unsigned short* p, bool rok, int kleft, bool vec,
                                            unsigned (&w)[8]) {
  if (rok && vec && kleft >= 16) {
    const u32x4 t0 = reinterpret_cast<const u32x4*>(p)[0];
    const u32x4 t1 = reinterpret_cast<const u32x4*>(p)[1];
    w[0] = t0.x; w[1] = t0.y; w[2] = t0.z; w[3] = t0.w;
    w[4] = t1.x; w[5] = t1.y; w[6] = t1.z; w[7] = t1.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned lo = (rok && 2 * j < kleft) ? p[2 * j] : 0u;
      const unsigned hi = (rok && 2 * j + 1 < kleft) ? p[2 * j + 1] : 0u;
      w[j] = lo | (hi << 16);
    }
  }
}

__device__ __forceinline__ void load_kcol16(const unsigned short* p, long long ld, bool rok, int kleft,
                                            unsigned (&w)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned lo = (rok && 2 * j < kleft) ? p[(long long)(2 * j) * ld] : 0u;
    const unsigned hi = (rok && 2 * j + 1 < kleft) ? p[(long long)(2 * j + 1) * ld] : 0u;
    w[j] = lo | (hi << 16);
  }
}

template <bool AM, bool BNC, typename S>
__global__ void __launch_bounds__(kThr, 2) gemm_x3_kernel(const GemmArgs a) {
  constexpr bool X3 = !is16<S>();
  constexpr int NP = X3 ? 2 : 1;                                     // LDS planes: hi (+ lo)
  __shared__ __attribute__((aligned(16))) u32x4 sA[2][NP * kBM * 4];   // [buf][plane][row][4]
  __shared__ __attribute__((aligned(16))) u32x4 sB[2][NP * kBN * 4];
  const S* Ap = static_cast<const S*>(a.A);
  const S* Bp = static_cast<const S*>(a.B);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wm = wave & 1;
  const int NT = (a.N + kBN - 1) / kBN;
  const int mt = blockIdx.x / NT, nt = blockIdx.x - mt * NT;
  const int m0 = mt * kBM, n0 = nt * kBN;
  const int split = blockIdx.y, bz = blockIdx.z;
  const int ksb = (a.K + kBK - 1) / kBK;          // K-steps per batch
  const int ktot = a.sum_b ? a.nb * ksb : ksb;
  const int kbeg = split * a.kps, kend = min(ktot, kbeg + a.kps);

  float sa = 1.f, sbs = 1.f;
  int ush = 0;
  if constexpr (X3) {
    const int ea = amax_exp(a.amax_a), eb = amax_exp(a.amax_b);
    sa = pow2f(kTop - ea);
    sbs = pow2f(kTop - eb);
    ush = ea + eb - 2 * kTop;
  }

  // staging roles: a K-contiguous operand takes (row = tid / 2, k half = tid & 1),
  // a row-contiguous one (row = tid & 127, k half = tid >> 7)
  const int ra = AM ? (tid & 127) : (tid >> 1), kha = AM ? (tid >> 7) * 16 : (tid & 1) * 16;
  const int rb = BNC ? (tid & 127) : (tid >> 1), khb = BNC ? (tid >> 7) * 16 : (tid & 1) * 16;
  const int ma = m0 + ra, nbr = n0 + rb;
  // fp32: 16 values per operand row segment; 16-bit: the same 16 as 8 packed pairs
  float va[X3 ? 16 : 1], vb[X3 ? 16 : 1];
  unsigned wa[X3 ? 1 : 8], wb[X3 ? 1 : 8];

  auto load = [&](int ks) __attribute__((always_inline)) {
    const int bb = a.sum_b ? ks / ksb : bz;
    const int k0 = (ks - (a.sum_b ? bb * ksb : 0)) * kBK;
    {
      const int kk = k0 + kha, kleft = a.K - kk;
      const bool rok = ma < a.M;
      const long long off = AM ? bb * a.sa + (long long)kk * a.lda + (rok ? ma : 0)
                               : bb * a.sa + (long long)(rok ? ma : 0) * a.lda + kk;
      if constexpr (X3) {
        const float* p = reinterpret_cast<const float*>(Ap) + off;
        if constexpr (AM) load_kcol(p, a.lda, rok, kleft, va);
        else load_krow(p, rok, kleft, a.vec_a, va);
        if (a.kmask_T) {
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if ((kk + j) % a.kmask_T == a.kmask_p) va[j] = 0.f;
        }
      } else {
        const unsigned short* p = reinterpret_cast<const unsigned short*>(Ap) + off;
        if constexpr (AM) load_kcol16(p, a.lda, rok, kleft, wa);
        else load_krow16(p, rok, kleft, a.vec_a, wa);
      }
    }
    {
      const int kk = k0 + khb, kleft = a.K - kk;
      const bool rok = nbr < a.N;
      const long long off = BNC ? bb * a.sb + (long long)kk * a.ldb + (rok ? nbr : 0)
                                : bb * a.sb + (long long)(rok ? nbr : 0) * a.ldb + kk;
      if constexpr (X3) {
        const float* p = reinterpret_cast<const float*>(Bp) + off;
        if constexpr (BNC) load_kcol(p, a.ldb, rok, kleft, vb);
        else load_krow(p, rok, kleft, a.vec_b, vb);
      } else {
        const unsigned short* p = reinterpret_cast<const unsigned short*>(Bp) + off;
        if constexpr (BNC) load_kcol16(p, a.ldb, rok, kleft, wb);
        else load_krow16(p, rok, kleft, a.vec_b, wb);
      }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      u32x4 H, L, HB, LB;
      if constexpr (X3) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned h, l;
          split_f16x2(va[8 * q + 2 * e], va[8 * q + 2 * e + 1], sa, h, l);
          H[e] = h; L[e] = l;
          split_f16x2(vb[8 * q + 2 * e], vb[8 * q + 2 * e + 1], sbs, h, l);
          HB[e] = h; LB[e] = l;
        }
      } else {
        H = (u32x4){wa[4 * q], wa[4 * q + 1], wa[4 * q + 2], wa[4 * q + 3]};
        HB = (u32x4){wb[4 * q], wb[4 * q + 1], wb[4 * q + 2], wb[4 * q + 3]};
      }
      const int ca = (kha / 8 + q) ^ swz(ra), cb = (khb / 8 + q) ^ swz(rb);
      sA[buf][ra * 4 + ca] = H;
      sB[buf][rb * 4 + cb] = HB;
      if constexpr (X3) {
        sA[buf][kBM * 4 + ra * 4 + ca] = L;
        sB[buf][kBN * 4 + rb * 4 + cb] = LB;
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lh = lane >> 5, lr = lane & 31, fsw = swz(lr);
  auto compute = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = (2 * ks + lh) ^ fsw;
      u32x4 wf[2][NP], af[2][NP];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          wf[i][p] = sB[buf][(p * kBN + wn * 64 + 32 * i + lr) * 4 + c];
          af[i][p] = sA[buf][(p * kBM + wm * 64 + 32 * i + lr) * 4 + c];
        }
      if constexpr (X3) {
#pragma unroll
        for (int t = 0; t < 3; ++t)   // hi*hi, hi*lo, lo*hi
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                  __builtin_bit_cast(f16x8, af[j][t == 1 ? 1 : 0]), __builtin_bit_cast(f16x8, wf[i][t == 2 ? 1 : 0]),
                  acc[j][i], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j][i] = mfma1<S>(af[j][0], wf[i][0], acc[j][i]);
      }
    }
  };

  if (kbeg < kend) {
    load(kbeg);
    store(0);
    __syncthreads();
    for (int ks = kbeg; ks < kend; ++ks) {
      const int cur = (ks - kbeg) & 1;
      const bool more = ks + 1 < kend;
      if (more) load(ks + 1);
      compute(cur);
      if (more) store(cur ^ 1);
      __syncthreads();
    }
  }

  // accumulator map (32x32x16, A fragments as the MFMA's rows): block (j, i) element
  // r2 is m = 32 j + 4 lh + (r2 & 3) + 8 (r2 >> 2), n = 32 i + lr, so each store
  // instruction writes two 128-B row segments
  const bool direct = a.splits == 1;
  const S* b0 = direct && a.bias0 ? static_cast<const S*>(a.bias0) + bz * a.sbias : nullptr;
  const S* b1 = direct && a.bias1 ? static_cast<const S*>(a.bias1) + bz * a.sbias : nullptr;
  S* outc = static_cast<S*>(a.C) + bz * a.sc;
  float* outs = a.slab + ((long long)bz * a.splits + split) * a.M * a.N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = n0 + wn * 64 + 32 * i + lr;
    if (n >= a.N) continue;
    float bias_n = 0.f;
    if (!a.bias_rows) {
      if (b0) bias_n += (float)b0[n];
      if (b1) bias_n += (float)b1[n];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        const int m = m0 + wm * 64 + 32 * j + 4 * lh + (r2 & 3) + 8 * (r2 >> 2);
        if (m >= a.M) continue;
        const float v = X3 ? __builtin_ldexpf(acc[j][i][r2], ush) : acc[j][i][r2];
        if (direct) {
          float bias = bias_n;
          if (a.bias_rows) {
            if (b0) bias += (float)b0[m];
            if (b1) bias += (float)b1[m];
          }
          outc[(long long)m * a.ldc + n] = (S)(v + bias);
        } else {
          outs[(long long)m * a.N + n] = v;
        }
      }
  }
}

// C[bz](m, n) = sum over splits in order + biases. grid covers nbz * M * N
template <typename S>
__global__ void __launch_bounds__(256) gemm_reduce_kernel(const GemmArgs a, long long total) {
  const long long mn = (long long)a.M * a.N;
  const S* b0 = static_cast<const S*>(a.bias0);
  const S* b1 = static_cast<const S*>(a.bias1);
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int bz = (int)(idx / mn);
    const long long r = idx - bz * mn;
    const int m = (int)(r / a.N), n = (int)(r - (long long)m * a.N);
    const float* s = a.slab + (long long)bz * a.splits * mn + r;
    float v = 0.f;
    for (int sp = 0; sp < a.splits; ++sp) v += s[sp * mn];
    const int bi = a.bias_rows ? m : n;
    if (b0) v += (float)b0[bz * a.sbias + bi];
    if (b1) v += (float)b1[bz * a.sbias + bi];
    static_cast<S*>(a.C)[bz * a.sc + (long long)m * a.ldc + n] = (S)v;
  }
}

// out[l][g] = sum_r x[l][r][g]: the rows in kColChunks consecutive chunks (each
// summed in row order), then the chunk partials in chunk order; with amax, also
// max |x| (atomicMax of the fp32 bit patterns into the zeroed slot), the scale
// source of the weight-gradient GEMMs that read x next.
constexpr int kColChunks = 64;
__device__ __forceinline__ long long col_rows(long long R) { return (R + kColChunks - 1) / kColChunks; }
__global__ void __launch_bounds__(256) colsum_part_kernel(const float* __restrict__ x, long long R, int G,
                                                          float* __restrict__ part, unsigned* amax) {
  const int g = blockIdx.x * 256 + threadIdx.x, ch = blockIdx.y, l = blockIdx.z;
  const long long rows = col_rows(R);
  const long long r0 = (long long)ch * rows, r1 = min(R, r0 + rows);
  float s = 0.f, m = 0.f;
  if (g < G) {
    const float* p = x + ((long long)l * R + r0) * G + g;
    long long r = r0;
    constexpr int U = 8;   // eight rows' loads in flight; the sum keeps row order
    for (; r + U <= r1; r += U, p += U * (long long)G) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[(long long)u * G];
#pragma unroll
      for (int u = 0; u < U; ++u) { s += v[u]; m = fmaxf(m, fabsf(v[u])); }
    }
    for (; r < r1; ++r, p += G) { s += *p; m = fmaxf(m, fabsf(*p)); }
    part[((long long)l * kColChunks + ch) * G + g] = s;
  }
  if (amax) {
    unsigned b = __builtin_bit_cast(unsigned, se::wave_max(m));
    if ((threadIdx.x & 63) == 0 && b) atomicMax(amax, b);
  }
}
__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ part, int G, int L,
                                                           float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L * G) return;
  const int l = i / G, g = i - l * G;
  const float* p = part + (long long)l * kColChunks * G + g;
  float s = 0.f;
#pragma unroll 8
  for (int c = 0; c < kColChunks; ++c) s += p[(long long)c * G];
  out[i] = s;
}

struct Plan {
  int MT, NT, nbz, ktot, splits, kps;
};

int plan_of(const se_gemm_desc* d, Plan& p) {
  if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batches <= 0) return SE_E_ARG;
  if (d->kmask_period < 0 || (d->kmask_period && (d->kmask_phase < 0 || d->kmask_phase >= d->kmask_period)))
    return SE_E_ARG;
  if (d->lda <= 0 || d->ldb <= 0 || d->ldc < d->N) return SE_E_ARG;
  p.MT = se::ceil_div(d->M, kBM);
  p.NT = se::ceil_div(d->N, kBN);
  if ((long long)p.MT * p.NT > 0x7fffffffLL) return SE_E_UNSUPPORTED;
  p.nbz = d->sum_batches ? 1 : d->batches;
  const int ksb = se::ceil_div(d->K, kBK);
  p.ktot = d->sum_batches ? d->batches * ksb : ksb;
  const long long tiles = (long long)p.MT * p.NT * p.nbz;
  int s = d->splits;
  if (s <= 0) {   // about two workgroups per CU, at least 16 K-steps per split
    s = 1;
    if (tiles < 512) s = (int)std::min<long long>((512 + tiles - 1) / tiles, std::max(1, p.ktot / 16));
  }
  s = std::max(1, std::min(s, p.ktot));
  p.kps = se::ceil_div(p.ktot, s);
  p.splits = se::ceil_div(p.ktot, p.kps);
  if (p.splits > 65535 || p.nbz > 65535) return SE_E_UNSUPPORTED;
  return SE_OK;
}

}  // namespace

extern "C" size_t se_gemm_workspace_size(const se_gemm_desc* d) {
  Plan p;
  if (plan_of(d, p) != SE_OK || p.splits == 1) return 0;
  return (size_t)p.nbz * p.splits * d->M * d->N * sizeof(float);
}

extern "C" int se_gemm(const se_gemm_desc* d, const void* A, const void* B, void* C, const void* bias0,
                       const void* bias1, const float* amax_a, const float* amax_b, void* ws, size_t ws_bytes,
                       void* stream) {
  Plan p;
  const int rc = plan_of(d, p);
  if (rc != SE_OK) return rc;
  const int dt = d->dtype;
  if (dt != SE_DTYPE_F32 && dt != SE_DTYPE_BF16 && dt != SE_DTYPE_F16) return SE_E_ARG;
  if (!A || !B || !C || (dt == SE_DTYPE_F32 && (!amax_a || !amax_b))) return SE_E_ARG;
  if (dt != SE_DTYPE_F32 && d->kmask_period) return SE_E_UNSUPPORTED;   // the masked form is fp32-only
  const size_t need = se_gemm_workspace_size(d);
  if (need && (!ws || ws_bytes < need)) return SE_E_WORKSPACE;
  GemmArgs a{};
  a.A = A; a.B = B; a.C = C; a.bias0 = bias0; a.bias1 = bias1; a.amax_a = amax_a; a.amax_b = amax_b;
  a.slab = (float*)ws;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c; a.sbias = d->stride_bias;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.nb = d->batches; a.sum_b = d->sum_batches ? 1 : 0;
  a.splits = p.splits; a.kps = p.kps;
  a.kmask_T = d->kmask_period; a.kmask_p = d->kmask_phase;
  a.bias_rows = d->bias_rows ? 1 : 0;
  // 16-B row loads: 4 fp32 / 8 16-bit elements per load, every row start 16-B aligned
  const int vq = dt == SE_DTYPE_F32 ? 4 : 8;
  a.vec_a = !d->a_mcontig && ((uintptr_t)A & 15) == 0 && d->lda % vq == 0 && d->stride_a % vq == 0;
  a.vec_b = !d->b_ncontig && ((uintptr_t)B & 15) == 0 && d->ldb % vq == 0 && d->stride_b % vq == 0;
  hipStream_t st = se::as_stream(stream);
  const dim3 grid(p.MT * p.NT, p.splits, p.nbz);
  const long long total = (long long)p.nbz * d->M * d->N;
  const long long blocks = std::min<long long>((total + 255) / 256, 4096);
#define SE_GEMM_LAUNCH(S)                                                                                          \
  do {                                                                                                             \
    if (d->a_mcontig) {                                                                                            \
      if (d->b_ncontig) hipLaunchKernelGGL((gemm_x3_kernel<true, true, S>), grid, dim3(kThr), 0, st, a);           \
      else hipLaunchKernelGGL((gemm_x3_kernel<true, false, S>), grid, dim3(kThr), 0, st, a);                       \
    } else {                                                                                                       \
      if (d->b_ncontig) hipLaunchKernelGGL((gemm_x3_kernel<false, true, S>), grid, dim3(kThr), 0, st, a);          \
      else hipLaunchKernelGGL((gemm_x3_kernel<false, false, S>), grid, dim3(kThr), 0, st, a);                      \
    }                                                                                                              \
    SE_LAUNCH_CHECK();                                                                                             \
    if (p.splits > 1) {                                                                                            \
      hipLaunchKernelGGL(gemm_reduce_kernel<S>, dim3((unsigned)blocks), dim3(256), 0, st, a, total);               \
      SE_LAUNCH_CHECK();                                                                                           \
    }                                                                                                              \
  } while (0)
  if (dt == SE_DTYPE_F32) SE_GEMM_LAUNCH(float);
  else if (dt == SE_DTYPE_BF16) SE_GEMM_LAUNCH(__bf16);
  else SE_GEMM_LAUNCH(_Float16);
#undef SE_GEMM_LAUNCH
  return SE_OK;
}

extern "C" size_t se_colsum_workspace_size(int L, long long R, int G) {
  if (L <= 0 || R <= 0 || G <= 0) return 0;
  return (size_t)L * kColChunks * G * sizeof(float);
}

extern "C" int se_colsum(const float* x, int L, long long R, int G, float* out, float* amax, void* ws,
                         size_t ws_bytes, void* stream) {
  if (!x || !out || L <= 0 || R <= 0 || G <= 0) return SE_E_ARG;
  if (L > 65535) return SE_E_UNSUPPORTED;
  if (!ws || ws_bytes < se_colsum_workspace_size(L, R, G)) return SE_E_WORKSPACE;
  hipStream_t st = se::as_stream(stream);
  if (amax && hipMemsetAsync(amax, 0, sizeof(float), st) != hipSuccess) return SE_E_LAUNCH;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(se::ceil_div(G, 256), kColChunks, L), dim3(256), 0, st, x, R, G,
                     (float*)ws, (unsigned*)amax);
  SE_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final_kernel, dim3(se::ceil_div((long long)L * G, 256)), dim3(256), 0, st,
                     (const float*)ws, G, L, out);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
