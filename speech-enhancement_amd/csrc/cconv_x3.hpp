// Split-bf16 ("bf16x3") variants of the conv GEMMs (included by cconv.hip,
// inside its anonymous namespace, after GatherArgs / xcd_remap).
//
// gfx950 has no TF32/xf32 MFMA: fp32-input MFMA (v_mfma_f32_32x32x2_f32) runs
// at the fp32 vector rate, 1/16 of the bf16 MFMA rate. Each fp32 operand is
// split into two bf16 terms, x = hi + lo + e with hi = bf16_rne(x),
// lo = bf16_rne(x - hi) (x - hi is exact in fp32), |e| <= 2^-17 |x|, and
//   a*b ~= ah*bh + ah*bl + al*bh        (dropped: al*bl, |.| <= 2^-16 |ab|)
// is accumulated in fp32 by three v_mfma_f32_32x32x16_bf16 (products of two
// bf16 are exact in the fp32 accumulator). Per-product error <= ~2^-15 |ab|,
// rms ~6e-6 |ab| on random data: fp32-class accuracy for the north star's
// 1e-4 relative bar at 3/16 of the fp32 MFMA cycles per FLOP.
//
// Operand lane map of v_mfma_f32_32x32x16_bf16: lane l (r = l & 31,
// h = l >> 5) holds A[row r][k = 8h + j] and B[k = 8h + j][col r] in element
// j. The accumulator map is the one of the fp32 32x32x2 form, so the
// epilogue is shared with gather_gemm_kernel.

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// (x0, x1) -> packed bf16 hi pair and lo pair (element 0 in the low half).
__device__ __forceinline__ void split_bf16x2(float x0, float x1, unsigned& hi, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0, x1}, bf16x2));
  const float h0 = __builtin_bit_cast(float, hi << 16);
  const float h1 = __builtin_bit_cast(float, hi & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0 - h0, x1 - h1}, bf16x2));
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}

// ---------------------------------------------------------------------------
// Scaled split-fp16 ("f16x3", SE_MATH_F16X3). fp16 keeps 11 significant bits
// (bf16: 8), so hi + lo carry 22 bits and the dropped lo*lo term is ~2^-22
// relative: fp32-class products at the cost of bf16x3. fp16's narrow exponent
// range is handled by a per-tensor power-of-two scale s = 2^(kF16Top - e),
// max|x| < 2^e, so every scaled value is below 2^14 (fp16 max 65504) and
// values down to 2^-17 max|x| keep a normal lo part. Scaling by a power of
// two is exact; the accumulator is multiplied back by 2^(ea + eb - 2 kF16Top)
// (v_ldexp_f32, exact) in the epilogue.
// ---------------------------------------------------------------------------
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
using se::kF16Top;
using se::amax_exp;
using se::pow2f;
using se::split_f16x2;

// one 32x32x16 MFMA on a pair of 16-B operand fragments: fp16 or bf16 elements
template <bool F16>
__device__ __forceinline__ f32x16 mfma_32x32x16(u32x4 a, u32x4 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                  c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                   c, 0, 0, 0);
}

// split of an operand pair into (hi, lo) planes: bf16, or scaled fp16
template <bool F16>
__device__ __forceinline__ void split2(float x0, float x1, float s, unsigned& hi, unsigned& lo) {
  if constexpr (F16) split_f16x2(x0, x1, s, hi, lo);
  else split_bf16x2(x0, x1, hi, lo);
}

// Per-tensor max |x| (SE_MATH_F16X3 scale source): atomic max of the fp32
// bit patterns (non-negative floats order as unsigned ints) into *out, which
// the caller zeroes first. Vectorised when x is 16-B aligned.
__global__ void __launch_bounds__(256) amax_kernel(const float* __restrict__ x, long long n, unsigned* out) {
  float m = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (((unsigned long long)x & 15) == 0) {
    const long long n4 = n >> 2;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    for (long long i = i0; i < n4; i += stride) {
      const f32x4 v = x4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    for (long long i = 4 * n4 + i0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  } else {
    for (long long i = i0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  }
  // (a NaN element is dropped by fmaxf; it still poisons the GEMM itself)
  unsigned b = __builtin_bit_cast(unsigned, m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned v = __shfl_xor(b, o);
    b = v > b ? v : b;
  }
  if ((threadIdx.x & 63) == 0 && b) atomicMax(out, b);
}

// LDS / pre-tiled weight image of one operand tile: [plane (hi, lo)][row][4
// chunks of 8 bf16 = 16 B], chunk c of row `row` stored at c ^ x3_swz(row).
// 64-B rows, XOR swizzle x3_swz = bit 2 of the row | (bit 1 ^ bit 4) << 1: the
// ds_read_b128 fragment reads (lane -> row r = l & 31, chunk 2ks + (l >> 5)) are
// conflict-free (in each lane group {0-3,12-15,20-27}, {4-11,16-19,28-31} the 16
// (row & 3, swizzle) pairs are distinct), and so are the activation tile's
// ds_write_b128 stores (8 consecutive rows of one 8-lane store group land on 8
// distinct 16-B slots of a 128-B bank row). Round 3: the (row >> 2) & 3 form left
// every store group 2-way conflicted (PMC: bank-conflict cycles 12-20 % of the
// LDS-array cycles of the gather GEMMs, tools/pmc_lds.sh).
__device__ __forceinline__ int x3_swz(int row) {
  return ((row >> 2) & 1) | ((((row >> 1) ^ (row >> 4)) & 1) << 1);
}
__device__ __forceinline__ int x3_chunk(int row, int c) { return c ^ x3_swz(row); }

constexpr int kX3BN = 128, kX3BM = 128;
// 32-k halves per staging round of the one-term gather tiles (SE_X3_HALVES=1: the
// round-3 32-k rounds, for A/B variant builds)
#ifndef SE_X3_HALVES
#define SE_X3_HALVES 2
#endif
constexpr int kX3OneTermHalves = SE_X3_HALVES;

// K order of the split GEMMs' weight image / ktab. kblk = 0: tap-major,
// k = tap * Cg + c. kblk = 32 (Cg % 32 == 0): channel-block-major, k =
// ((c / 32) * taps + tap) * 32 + c % 32, so a tile visits every tap of a
// 32-channel block in consecutive K-steps and the block's input rows are
// re-read from L2 instead of after a sweep over all Cg channels (which
// evicts them). ktab[k].w holds the channel c.
__device__ __forceinline__ void split_k(int k, int Cg, int ntaps, int kblk, int& t, int& c) {
  if (kblk) {
    const int s = k / kblk, cl = k - s * kblk;
    t = s % ntaps;
    c = (s / ntaps) * kblk + cl;
  } else {
    t = k / Cg;
    c = k - t * Cg;
  }
}
constexpr int kX3TileU4 = 2 * 128 * 4;   // u32x4 per (k-step, n-tile) weight image = 16 KB

// Pre-tiled split weight: Wt[(s * NT + t) * kX3TileU4 + (plane * 128 + n) * 4 + x3_chunk(n, c)]
// holds bf16 element e of k = 32 s + 8 c + e, column n0 = 128 t + n. Also ktab
// (as prep_class_kernel).
// F16: scaled split-fp16 planes (amax_w = max |weight|, see amax_exp)
template <bool F16 = false>
__global__ void prep_class_x3_kernel(WeightView w, TapList taps, int Cg, int N, int Kp, int NT,
                                     int Hi, int Wi, int data_grad, int kblk, unsigned short* Wt,
                                     int4* ktab, const float* amax_w) {
  const int K = taps.n * Cg;
  const float sw = (F16 && amax_w) ? pow2f(kF16Top - amax_exp(amax_w)) : 1.f;   // no bound: unscaled (SE_MATH_F16)
  const long long total = (long long)Kp * NT * 128;   // one thread per (k, n)
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(idx % Kp);                    // k fastest: a thread group fills rows
    const int n = (int)(idx / Kp);
    float v = 0.f;
    if (k < K && n < N) {
      int t, c;
      split_k(k, Cg, taps.n, kblk, t, c);
      const int ci = data_grad ? n : c, co = data_grad ? c : n;
      v = kernel_value(w, ci, co, taps.ti[t], taps.tj[t]);
    }
    unsigned short hb, lb;
    if constexpr (F16) {
      const float vs = v * sw;
      const _Float16 h16 = (_Float16)vs;
      hb = __builtin_bit_cast(unsigned short, h16);
      lb = __builtin_bit_cast(unsigned short, (_Float16)(vs - (float)h16));
    } else {
      const float h = (float)(__bf16)v;
      hb = bf16_bits(v);
      lb = bf16_bits(v - h);
    }
    const int s = k >> 5, kc = (k >> 3) & 3, e = k & 7;
    const int tn = n >> 7, nl = n & 127;
    const long long base = ((long long)s * NT + tn) * kX3TileU4 * 8;   // in bf16 units
    const long long off = ((long long)nl * 4 + x3_chunk(nl, kc)) * 8 + e;
    Wt[base + off] = hb;
    Wt[base + 128 * 4 * 8 + off] = lb;
    if (n == 0) {
      int4 q;
      q.w = 0;
      if (k < K) {
        int t, c;
        split_k(k, Cg, taps.n, kblk, t, c);
        q.x = (int)((long long)c * Hi * Wi + (long long)taps.offh[t] * Wi + taps.offw[t]);
        q.y = taps.offh[t];
        q.z = taps.offw[t];
        q.w = c;
      } else {
        q.x = 0; q.y = kInvalidOff; q.z = 0;
      }
      ktab[k] = q;
    }
  }
}

// Gather GEMM, split-bf16: same contraction, tiling and epilogue as
// gather_gemm_kernel<128, 128, 2, 2, TU>. a.Wp points at the pre-tiled split
// weight (prep_class_x3_kernel), a.ldw = 128 * gridDim.y.
// Per K-step (BK = 32) a wave issues 2 k-substeps x 2 x 2 blocks x 3 terms =
// 24 MFMAs of 32 cycles; each thread gathers 16 consecutive k of one m column
// (k = k0 + 16 * akr + j), splits them in registers and writes 4 ds_write_b128.
// TERMS = 1 is the plain bf16 GEMM (SE_MATH_BF16: operands rounded to bf16,
// fp32 accumulate, the arithmetic of autocast's bf16 conv): only the hi planes
// are staged and read.
// JM: decoder skip join (GatherArgs::X2 / Y2): 0 none, 1 the gathered tensor
// is the joined input (forward), 2 the output is split into the joined
// input's two gradients (data-grad). Both need the TU path.
// NW: 128-column weight tiles per workgroup. NW = 2 is a 256 (n) x 128 (m)
// tile of 8 waves (one workgroup per CU): each gathered activation is loaded
// and split once per 256 output columns instead of once per 128.
// F16: scaled split-fp16 operands (SE_MATH_F16X3; a.amax_a / a.amax_w give the
// per-tensor scales of the gathered tensor and the weights).
// SD: storage type of X and Y (se_conv2d_desc.dtype): 0 fp32; 1 bf16 / 2 fp16 with
// the one-term MFMA of that format (TERMS = 1; F16 = fp16 MFMA, unscaled: the
// operands are exactly representable), the 16-bit tensors loaded and stored as they are.
template <bool TU, int TERMS = 3, int JM = 0, int NW = 1, bool F16 = false, int SD = 0>
__global__ void __launch_bounds__(kThreads * NW, NW == 1 ? 2 : 1)
gather_x3_kernel(const GatherArgs a) {
  static_assert(TERMS == 1 || TERMS == 3, "hi*hi, or hi*hi + hi*lo + lo*hi");
  static_assert(SD == 0 || TERMS == 1, "16-bit storage: one-term tiles");
  static_assert(SD == 0 || F16 == (SD == 2), "16-bit storage: the MFMA format is the storage format");
  static_assert(JM == 0 || TU, "the joined gather / epilogue run on the tap-uniform path");
  constexpr int ES = SD ? 2 : 4;                  // bytes per element of X / Y
  static_assert(NW == 1 || NW == 2, "128 or 256 columns per workgroup");
  constexpr int PL = TERMS == 1 ? 1 : 2;          // operand planes staged / read
  constexpr int THR = kThreads * NW;
  constexpr int BN = kX3BN * NW, BM = kX3BM, WM = 2, TN = 64, TM = 64, RN = 2, RM = 2;
  constexpr int AJ = 16 / NW;                     // gathered k per thread per 32-k half
  constexpr int CPT = AJ / 8;                     // 16-B chunks per plane per thread
  // 32-k halves per staging round: one term stages two (BK = 64; the lo-plane LDS
  // slots hold the second half), so a barrier feeds 16 MFMAs per wave, not 8
  constexpr int KH = TERMS == 1 ? kX3OneTermHalves : 1;
  constexpr int BKS = kBK * KH;
  __shared__ __attribute__((aligned(16))) u32x4 sA[2][2 * BM * 4];
  __shared__ __attribute__((aligned(16))) u32x4 sW[2][2 * BN * 4];   // [t][plane][128 rows][4]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int NT = gridDim.y;                       // workgroup column tiles (BN wide)
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const long long HiWi = (long long)a.Hi * a.Wi;

  const int am = tid % BM;
  const int akr = __builtin_amdgcn_readfirstlane(tid / BM);   // 0 .. 2 NW - 1 (wave-uniform)
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
  float sa = 1.f;   // F16 (three terms): activation scale; the epilogue multiplies by 2^ush
  int ush = 0;
  if constexpr (F16 && TERMS == 3) {
    const int ea = amax_exp(a.amax_a);
    sa = pow2f(kF16Top - ea);
    ush = ea + amax_exp(a.amax_w) - 2 * kF16Top;
  }
  struct Stage { typename StageT<SD>::T ra[AJ * KH]; u32x4 rw[2 * PL * KH]; };   // 16-bit storage: raw bits
  Stage s0, s1;
  using se::uniform_ptr;
  const int b0 = m0 / (a.Qh * a.Qw);
  const int cpb = JM == 1 ? 2 * a.jh : a.Cg;      // channels per batch item of X
  const long long H2W2 = (long long)a.H2 * a.W2;
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr((const char*)a.X + (long long)b0 * cpb * HiWi * ES), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rx2 = rx;
  if constexpr (JM == 1)
    rx2 = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr((const char*)a.X2 + (long long)b0 * cpb * H2W2 * ES), (short)0,
                                            0x7FFFFFFF, 0x00020000);
  // this workgroup's NW consecutive 128-column images of one k-step; a
  // thread's element e = tid + THR j (j < 2 PL) of [t][plane][row][4]; with
  // one plane (PL = 1) the lo planes are skipped
  const u32x4* wt = reinterpret_cast<const u32x4*>(a.Wp) + (long long)nt * NW * kX3TileU4;
  int xoff = 0, xoff2 = 0;
  if constexpr (TU) {
    if (mval) {
      const int b = m / (a.Qh * a.Qw);
      xoff = (int)(((long long)(b - b0) * cpb * HiWi + (long long)hb * a.Wi + wb) * ES);
      if constexpr (JM == 1) xoff2 = (int)(((long long)(b - b0) * cpb * H2W2 + (long long)hb * a.W2 + wb) * ES);
    }
  }
  auto load_tile = [&](Stage& st, int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      const int kh0 = k0 + kBK * h;
      if constexpr (TU) {
        const int4 e0 = a.ktab[kh0];              // the half's tap and first channel (uniform)
        int c0 = e0.w;
        const int hi = hb + e0.y, wi = wb + e0.z;
        bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
        int vo = xoff + (e0.y * a.Wi + e0.z) * ES, cs = (int)(HiWi * ES);
        __amdgpu_buffer_rsrc_t r = rx;
        if constexpr (JM == 1) {                  // a K-step lies in one join chunk
          // chunks [x_re, s_re, x_im, s_im] (complex_concat), or [x_re, x_im, s_re, s_im]
          // (torch.cat, a.jcat: DCUNet's decoder, _1903_03107_dcunet.py:93)
          const int q = c0 / a.jh;
          const bool from_x = a.jcat ? q < 2 : (q & 1) == 0;
          c0 = (a.jcat ? (q & 1) : (q >> 1)) * a.jh + (c0 - q * a.jh);
          ok &= !from_x | ((hi < a.H2) & (wi < a.W2));   // F.pad rows / columns of x read 0
          vo = from_x ? xoff2 + (e0.y * a.W2 + e0.z) * ES : vo;
          cs = from_x ? (int)(H2W2 * ES) : cs;
          r = from_x ? rx2 : rx;
        }
        vo = ok ? vo : (int)0x80000000;
        c0 += AJ * akr;
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
          if constexpr (SD != 0) st.ra[AJ * h + j] = bload_raw16(r, vo, (c0 + j) * cs);
          else st.ra[AJ * h + j] = bload<0>(r, vo, (c0 + j) * cs);
        }
      } else {
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
          const int4 e = a.ktab[kh0 + AJ * akr + j];   // uniform index -> s_load
          const int hi = hb + e.y, wi = wb + e.z;
          const bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
          const void* src = ok ? (const void*)a.X : (const void*)a.zero;
          if constexpr (SD != 0) st.ra[AJ * h + j] = ld_raw16(src, ok ? xbase + e.x : 0);
          else st.ra[AJ * h + j] = ld_s<0>(src, ok ? xbase + e.x : 0);
        }
      }
      const u32x4* src = wt + (long long)((kh0 >> 5)) * NT * NW * kX3TileU4;
#pragma unroll
      for (int j = 0; j < 2 * PL; ++j) {
        const int e = tid + THR * j;
        st.rw[2 * PL * h + j] = src[PL == 2 ? e : e + (e >> 9) * 512];
      }
    }
  };
  const int swz = x3_swz(am);
  auto store_tile = [&](const Stage& st, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int hk = 0; hk < KH; ++hk) {            // one term: half hk in the plane-hk slots
#pragma unroll
      for (int q = 0; q < CPT; ++q) {
        u32x4 H, L;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i0 = AJ * hk + 8 * q + 2 * e;
          unsigned h, l = 0;
          if constexpr (SD != 0) h = st.ra[i0] | (st.ra[i0 + 1] << 16);   // = split2's hi, sa = 1
          else split2<F16>(st.ra[i0], st.ra[i0 + 1], sa, h, l);
          H[e] = h;
          L[e] = l;
        }
        const int c = (CPT * akr + q) ^ swz;
        sA[buf][hk * BM * 4 + am * 4 + c] = H;
        if constexpr (PL == 2) sA[buf][BM * 4 + am * 4 + c] = L;
      }
#pragma unroll
      for (int j = 0; j < 2 * PL; ++j) sW[buf][hk * BN * 4 + tid + THR * j] = st.rw[2 * PL * hk + j];
    }
  };

  f32x16 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lh = lane >> 5, lr = lane & 31;
  const int fsw = x3_swz(lr);
  // both k-substeps' fragments are read up front
  auto compute = [&](int cur) __attribute__((always_inline)) {
    u32x4 wf[KH][2][RN][PL], af[KH][2][RM][PL];     // [half][ks][block][plane]
#pragma unroll
    for (int hk = 0; hk < KH; ++hk)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = (2 * kk + lh) ^ fsw;
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          const int n = wn * TN + 32 * i;       // block's first column (uniform)
#pragma unroll
          for (int p = 0; p < PL; ++p)
            wf[hk][kk][i][p] = sW[cur][hk * BN * 4 + (((n >> 7) * PL + p) * 128 + (n & 127) + lr) * 4 + c];
        }
#pragma unroll
        for (int j = 0; j < RM; ++j)
#pragma unroll
          for (int p = 0; p < PL; ++p)
            af[hk][kk][j][p] = sA[cur][((p + hk) * BM + wm * TM + 32 * j + lr) * 4 + c];
      }
#pragma unroll
    for (int hk = 0; hk < KH; ++hk)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int t = 0; t < TERMS; ++t)  // terms: hi*hi, hi*lo, lo*hi
#pragma unroll
          for (int i = 0; i < RN; ++i)
#pragma unroll
            for (int j = 0; j < RM; ++j)
              acc[i][j] = mfma_32x32x16<F16>(wf[hk][kk][i][t == 2 ? 1 : 0], af[hk][kk][j][t == 1 ? 1 : 0], acc[i][j]);
  };
  // one scheduling region per K-step: the non-MFMA stream (next tiles' loads,
  // fragment reads, LDS writes) interleaved into the MFMA gaps
#ifndef SE_X3_SCHED
#define SE_X3_SCHED 0   // variant builds: 1 = two DS / two VALU per MFMA, 2 = the global loads first
#endif
  auto interleave = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);                  // first fragments
    if constexpr (SE_X3_SCHED == 2) __builtin_amdgcn_sched_group_barrier(0x020, (AJ + 2 * PL) * KH, 0);
#pragma unroll
    for (int i = 0; i < 2 * TERMS * RN * RM * KH; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                // MFMA
      __builtin_amdgcn_sched_group_barrier(0x080, SE_X3_SCHED == 1 ? 2 : 1, 0);   // DS
      if (SE_X3_SCHED != 2 && i < (AJ + 2 * PL) * KH) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // global load
      __builtin_amdgcn_sched_group_barrier(0x002, SE_X3_SCHED == 1 ? 2 : 3, 0);   // VALU
    }
  };

  const int nk = a.Kp / BKS;   // one term: Kp % 64 == 0 (plan_pass)
  // two register staging sets (prefetch distance 2); unconditional (clamped) loads and
  // stores keep each step one scheduling region: a clamped reload of the last tile
  // lands in the buffer no step reads
  load_tile(s0, 0);
  store_tile(s0, 0);
  if (nk > 1) load_tile(s1, BKS);
  __syncthreads();
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    load_tile(s0, min(kt + 2, nk - 1) * BKS);
    compute(0);
    store_tile(s1, 1);
    interleave();
    __syncthreads();
    load_tile(s1, min(kt + 3, nk - 1) * BKS);
    compute(1);
    store_tile(s0, 0);
    interleave();
    __syncthreads();
  }
  if (kt < nk) compute(0);
  if constexpr (F16 && TERMS == 3) {   // undo the operand scales (exact)
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int j = 0; j < RM; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], ush);
  }

  // --- epilogue (as gather_gemm_kernel) ---
  __syncthreads();
  float* sBias = reinterpret_cast<float*>(&sW[0][0]);
  for (int i = tid; i < BN; i += THR) {
    const int n = n0 + i;
    sBias[i] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
  }
  __syncthreads();
  const long long HoWo = (long long)a.Ho * a.Wo;
  const bool full_n = n0 + BN <= a.N;
  // accumulator map: block (i, j) element r2 is column (m) 32 j + lr and row
  // (n) 32 i + 4 lh + (r2 & 3) + 8 (r2 >> 2) of the wave tile
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const int mm = m0 + wm * TM + 32 * j + lr;
    if (mm >= a.M) continue;
    const int qhw = a.Qh * a.Qw;
    const int b = mm / qhw, r = mm - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    const int nl0 = wn * TN + 4 * lh;
    if constexpr (JM == 2) {
      // joined output: a 32-row block of n lies in one join chunk (yjh % 32 == 0);
      // s chunks -> Y over Ho x Wo, x chunks -> Y2 over YH2 x YW2 (rows >= YH2 and, for a
      // padded x (a.jcat), columns >= YW2 are the F.pad zeros: no x gradient)
      const int oh = a.ph + a.Sh * qh, ow = a.pw + a.Sw * qw;
      const long long P2 = (long long)a.YH2 * a.YW2;
      const int cpb = 2 * a.yjh;
#pragma unroll
      for (int i = 0; i < RN; ++i) {
        const int nb = n0 + wn * TN + 32 * i;     // block's first channel (wave-uniform)
        const int q = nb / a.yjh;
        const int cb = (a.jcat ? (q & 1) : (q >> 1)) * a.yjh + (nb - q * a.yjh) + 4 * lh;
        const bool to_x = a.jcat ? q < 2 : (q & 1) == 0;
        if (to_x && (oh >= a.YH2 || ow >= a.YW2)) continue;
        const long long pl = to_x ? P2 : HoWo;
        const long long yo = to_x ? ((long long)b * cpb + cb) * P2 + (long long)oh * a.YW2 + ow
                                  : ((long long)b * cpb + cb) * HoWo + (long long)oh * a.Wo + ow;
        void* yb = to_x ? (void*)a.Y2 : (void*)a.Y;
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) st_s<SD>(yb, yo + (long long)((r2 & 3) + 8 * (r2 >> 2)) * pl, acc[i][j][r2]);
      }
      continue;
    }
    const long long yb = (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo +
                         (a.pw + a.Sw * qw) + (long long)(n0 + nl0) * HoWo;
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        const int nl = 32 * i + (r2 & 3) + 8 * (r2 >> 2);
        if (full_n || n0 + nl0 + nl < a.N) st_s<SD>(a.Y, yb + (long long)nl * HoWo, acc[i][j][r2] + sBias[nl0 + nl]);
      }
  }
}

// ---------------------------------------------------------------------------
// Weight-grad reduction GEMM, split-bf16: dWp[k, n] = sum_m G[m, k] * D[m, n]
// over one m-split per workgroup (same slabs / finish path as
// wgrad_gemm_kernel<128, 128, 2, 2, 32, TU>).
// The reduction index m is the MFMA k: a step of BMR = 32 positions is two
// 16-deep k-substeps. Lanes load along m (coalesced along time); a half-wave
// owns 16 consecutive G rows and 16 consecutive D rows, so a thread holds, per
// position, 16 consecutive rows = two 16-B chunks of a [position][row] LDS
// image (hi and lo planes). The MFMA fragments (row = lane, 8 positions) are
// read back transposed with ds_read_b64_tr_b16 (gfx950), two per fragment.
// Image rows are 256 B (128 bf16) with the XOR chunk swizzle below, which
// keeps both the transposed reads and the b128 stores (nearly) conflict-free.
// ---------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// chunk swizzle of position row s (an involution on the 16 chunks)
__device__ __forceinline__ int wx3_swz(int s) {
  // bits 2-3 = s & 3 keep the transposed reads conflict-free (4 consecutive positions x 4
  // chunks on 16 distinct 16-B slots); bits 0-2 = (s1, s2, s0) put 8 consecutive positions
  // of one ds_write_b128 store group on 8 distinct slots (the round-2 form (s >> 2) & 3 was
  // 2-way: a third of the weight-grads' LDS-array cycles, tools/pmc_lds.sh)
  return ((s & 3) << 2) | (((s >> 2) & 1) << 1) | ((s >> 1) & 1);
}
__device__ __forceinline__ int wx3_off(int s, int ch) {   // byte offset of chunk ch of position row s
  return 256 * s + 16 * (ch ^ wx3_swz(s));
}

// DJ: D is the decoder skip join (WgradArgs::D2, a transposed conv's input).
// F16: scaled split-fp16 operands (SE_MATH_F16X3; a.amax_g / a.amax_d).
// NB: 128-row D blocks per workgroup (tile 128 k x 128 NB n, 4 NB waves of
// 64 x 64). With NB = 2 the gathered G tile of a step is loaded and split once
// for 256 output columns (a thread stages 8 G rows and 16 D rows instead of
// 16 + 16), a quarter fewer loads and splits per MFMA; every output keeps its
// m-split and its order of positions, so the slabs are bit-identical.
// KP: the K range ends inside the last k-tile (ntaps * Cg % 128 != 0).
// SD: storage type of X / D (as gather_x3_kernel; 16-bit with the one-term MFMA)
// KB: 128-row G blocks per workgroup (KB = 2 with NB = 2: 256 k x 256 n tiles, 8 waves of
// 128 x 64, one register staging set; a staged G row serves 256 columns and a staged D
// row 256 k rows, a third fewer loads and splits per MFMA than 128 x 256. KB = 2 with
// NB = 1 (round 6): 256 k x 128 n, 8 waves of 64 x 64 for N = 128 (the encoder): two taps
// per workgroup share each staged dy row)
template <bool TU, int TERMS = 3, bool DJ = false, bool F16 = false, int NB = 1, bool KP = false, int SD = 0,
          int KB = 1>
__global__ void __launch_bounds__(NB == 2 || KB == 2 ? 2 * kThreads : kThreads, 2)
wgrad_x3_kernel(const WgradArgs a) {
  static_assert(TERMS == 1 || TERMS == 3, "hi*hi (SE_MATH_BF16), or hi*hi + hi*lo + lo*hi");
  static_assert(SD == 0 || TERMS == 1, "16-bit storage: one-term tiles");
  static_assert(SD == 0 || F16 == (SD == 2), "16-bit storage: the MFMA format is the storage format");
  constexpr int ES = SD ? 2 : 4;             // bytes per element of X / D
  static_assert(NB == 1 || NB == 2, "one or two 128-row D blocks");
  static_assert(KB == 1 || (KB == 2 && !KP), "256-row G tiles: full K");
  constexpr int PL = TERMS == 1 ? 1 : 2;     // planes staged / read per operand
  // waves: 4 (128 x 128) or 8 (128 x 256, 256 x 256)
  constexpr int NWV = NB == 2 || KB == 2 ? 8 : 4, THR = 64 * NWV;
  constexpr int BKO = 128 * KB, BNO = 128 * NB, WNn = 2 * NB, TK = BKO * WNn / NWV, TN = 64, RK = TK / 32, RN = 2;
  constexpr int BMR = 32;
  constexpr int DWR = BNO / NWV;             // D rows per wave
  constexpr int RJ = DWR / 2;                // D rows per thread
  constexpr int GW = BKO / NWV;              // G rows per wave
  constexpr int RJG = GW / 2;                // G rows per thread
  constexpr int PLANE = BMR * 256;           // bytes of one [32 positions][128 rows] bf16 plane
  // per 128-row G block: G hi, G lo; then per 128-row D block: D hi, D lo
  constexpr int DPL = 2 * KB;                // first D plane
  // 32-position halves per staging round: one term stages two (64 positions; the lo
  // plane slots hold the second half), so a barrier feeds 16 MFMAs per wave, not 8;
  // the positions are accumulated in the same order, so the slabs are unchanged
  constexpr int KH = TERMS == 1 && KB == 1 ? kX3OneTermHalves : 1;   // 256 x 256: one half (registers)
  __shared__ __attribute__((aligned(16))) unsigned char sm[2][(2 * KB + 2 * NB) * PLANE];
  __shared__ int4 sK[BKO];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave / WNn, wnn = wave % WNn;
  // tile space (a.vk k-tiles x a.vn n-tiles x a.vs m-splits), walked by a 1-D
  // grid of at most that many workgroups (a persistent grid when capped)
  const int nkn = a.vk * a.vn, ntiles = nkn * a.vs;
  for (int L = blockIdx.x; L < ntiles; L += gridDim.x) {
  const int tile = xcd_remap(L, ntiles);
  const int split = tile / nkn, kn = tile % nkn;
  const int k0 = (kn % a.vk) * BKO, n0 = (kn / a.vk) * BNO;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const long long HiWi = (long long)a.Hi * a.Wi;
  const long long QQ = (long long)a.Qh * a.Qw;
  const int ml = lane & 31, lr = lane >> 5;
  // valid k rows of this tile (k < ntaps * Cg; the rest is Kp padding, e.g.
  // 108 of 128 in a first conv with Cg = 2): a wave skips the loads, splits,
  // fragment reads and MFMAs of 32-row blocks that hold only padding (their
  // slab rows stay 0), wave-uniform; only in the KP instantiation (the branches
  // cost the full tiles their MFMA interleave: 627 vs 629 utt/s when always on)
  const int kv = KP ? min(BKO, a.ntaps * a.Cg - k0) : BKO;
  const int kvw = kv - wk * TK;                       // ... of this wave's 64 MFMA rows
  const bool gact = GW * wave < kv;                   // this wave stages some valid G row
  const int rbase = DWR * wave + RJ * lr;    // this thread's first D row
  const int rbase_g = GW * wave + RJG * lr;  // ... and first G row

  for (int i = tid; i < BKO; i += THR) sK[i] = a.ktab ? a.ktab[k0 + i] : wgrad_ktab(a, k0 + i);
  __syncthreads();
  float sg = 1.f, sd = 1.f;   // F16 (three terms): operand scales; the slab gets acc * 2^ush
  int ush = 0;
  if constexpr (F16 && TERMS == 3) {
    const int eg = amax_exp(a.amax_g), ed = amax_exp(a.amax_d);
    sg = pow2f(kF16Top - eg);
    sd = pow2f(kF16Top - ed);
    ush = eg + ed - 2 * kF16Top;
  }

  int cb, cqh, cqw;
  {
    const long long mm = mbeg + ml;
    cb = (int)(mm / QQ);
    const int r = (int)(mm - cb * QQ);
    cqh = r / a.Qw;
    cqw = r - cqh * a.Qw;
  }
  struct Stage { typename StageT<SD>::T rg[RJG * KH], rd[RJ * KH]; };   // 16-bit: raw bits
  Stage st0, st1;
  using se::uniform_ptr;
  const int bfirst = (int)(mbeg / QQ);
  __amdgpu_buffer_rsrc_t rg_src = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr((const char*)a.X + (long long)bfirst * a.Cg * HiWi * ES), (short)0, 0x7FFFFFFF, 0x00020000);
  const int dcpb = DJ ? 2 * a.djh : a.N;         // channels per batch item of D
  const long long QQ2 = (long long)a.DH2 * a.DW2;
  __amdgpu_buffer_rsrc_t rd_src = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr((const char*)a.D + (long long)bfirst * dcpb * QQ * ES), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rd2_src = rd_src;
  if constexpr (DJ)
    rd2_src = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr((const char*)a.D2 + (long long)bfirst * dcpb * QQ2 * ES), (short)0,
                                                0x7FFFFFFF, 0x00020000);
  const int4 tap_e = sK[rbase_g & ~127];           // TU: one tap per 128-row G block
  const int cbase = (k0 + (rbase_g & ~127)) % a.Cg;
  const bool one_wrap = a.Qw >= BMR;
  auto advance1 = [&](int& b_, int& h_, int& w_) __attribute__((always_inline)) {
    if (one_wrap) {
      w_ += BMR;
      const bool w1 = w_ >= a.Qw;
      w_ -= w1 ? a.Qw : 0;
      h_ += w1 ? 1 : 0;
      const bool w2 = h_ >= a.Qh;
      h_ = w2 ? 0 : h_;
      b_ += w2 ? 1 : 0;
    } else {
      const int t = w_ + BMR;
      const int dq = t / a.Qw;
      w_ = t - dq * a.Qw;
      const int u = h_ + dq;
      const int db = u / a.Qh;
      h_ = u - db * a.Qh;
      b_ += db;
    }
  };
  auto advance = [&]() __attribute__((always_inline)) { advance1(cb, cqh, cqw); };
  auto load_step = [&](Stage& S, int mstep0) __attribute__((always_inline)) {
#pragma unroll
   for (int hh = 0; hh < KH; ++hh) {
    const int mstep = mstep0 + BMR * hh;
    const bool mv = mstep + ml < mend;
    const int rb = cb - bfirst;
    // D rows of this thread: n0 + rbase + j, j < RJ. The host runs this kernel
    // only for N % 16 == 0, so a thread's rows are all inside N or all in the
    // Np-padded tail; tail rows read 0 through an out-of-range voffset (they
    // must not be read: past the last batch item they leave the allocation).
    const bool dok = mv & (n0 + rbase < a.N);
    int vd, ds = (int)(QQ * ES), srow = DWR * wave;
    __amdgpu_buffer_rsrc_t rdr = rd_src;
    if constexpr (DJ) {
      // joined D: chunks [x_re, s_re, x_im, s_im] (complex_concat) or [x_re, x_im, s_re,
      // s_im] (torch.cat, a.djcat) of djh rows; a wave's 32 rows lie in one chunk
      // (djh % 32 == 0)
      const int nb = n0 + DWR * wave;
      const int q = nb / a.djh;
      const bool from_x = a.djcat ? q < 2 : (q & 1) == 0;
      const int cr = (a.djcat ? (q & 1) : (q >> 1)) * a.djh + (nb - q * a.djh) + RJ * lr;   // row in its source
      const bool okx = dok & (!from_x | ((cqh < a.DH2) & (cqw < a.DW2)));   // F.pad rows / columns of x: 0
      vd = from_x ? (int)(((long long)rb * dcpb * QQ2 + (long long)cr * QQ2 + (long long)cqh * a.DW2 + cqw) * ES)
                  : (int)(((long long)rb * dcpb * QQ + (long long)cr * QQ + (long long)cqh * a.Qw + cqw) * ES);
      vd = okx ? vd : (int)0x80000000;
      ds = from_x ? (int)(QQ2 * ES) : ds;
      rdr = from_x ? rd2_src : rd_src;
      srow = 0;
    } else {
      vd = dok ? (int)(((long long)rb * a.N * QQ + (long long)(n0 + RJ * lr) * QQ +
                        (long long)cqh * a.Qw + cqw) * ES) : (int)0x80000000;
    }
    if (KP && !gact) {
#pragma unroll
      for (int j = 0; j < RJG; ++j) S.rg[RJG * hh + j] = 0.f;
    } else if constexpr (TU) {
      const int hi = cqh * a.sh + tap_e.y, wi = cqw * a.sw + tap_e.z;
      const bool ok = mv & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      const int vg = ok ? (int)(((long long)rb * a.Cg * HiWi + (long long)(cbase + RJG * lr) * HiWi +
                                 (long long)hi * a.Wi + wi) * ES) : (int)0x80000000;
      const int gs = (int)(HiWi * ES);
#pragma unroll
      for (int j = 0; j < RJG; ++j) {
        if constexpr (SD != 0) S.rg[RJG * hh + j] = bload_raw16(rg_src, vg, (((GW * wave) & 127) + j) * gs);
        else S.rg[RJG * hh + j] = bload<0>(rg_src, vg, (((GW * wave) & 127) + j) * gs);
      }
    } else {
      const int hb = cqh * a.sh, wb = cqw * a.sw;
      const long long xb = (long long)cb * a.Cg * HiWi + (long long)hb * a.Wi + wb;
#pragma unroll
      for (int j = 0; j < RJG; ++j) {
        const int4 e = sK[rbase_g + j];
        const int hi = hb + e.y, wi = wb + e.z;
        const bool ok = mv & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
        const void* src = ok ? (const void*)a.X : (const void*)a.zero;
        if constexpr (SD != 0) S.rg[RJG * hh + j] = ld_raw16(src, ok ? xb + e.x : 0);
        else S.rg[RJG * hh + j] = ld_s<0>(src, ok ? xb + e.x : 0);
      }
    }
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
      if constexpr (SD != 0) S.rd[RJ * hh + j] = bload_raw16(rdr, vd, (srow + j) * ds);
      else S.rd[RJ * hh + j] = bload<0>(rdr, vd, (srow + j) * ds);
    }
    advance();
   }
  };
  auto store_step = [&](const Stage& S, int buf) __attribute__((always_inline)) {
   unsigned char* base = sm[buf];
#pragma unroll
   for (int hh = 0; hh < KH; ++hh) {   // one term: half hh in the plane-hh slots
    unsigned char* dbase = base + (DPL + 2 * (rbase >> 7) + hh) * PLANE;   // this thread's D block
    unsigned char* gbase = base + (2 * (rbase_g >> 7) + hh) * PLANE;      // ... and G block
#pragma unroll
    for (int q = 0; q < (RJG > RJ ? RJG : RJ) / 8; ++q) {
      u32x4 GH, GL, DH, DL;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned h, l = 0;
        if (q < RJG / 8) {
          const int ig = RJG * hh + 8 * q + 2 * e;
          if constexpr (SD != 0) h = S.rg[ig] | (S.rg[ig + 1] << 16);   // split2's hi, sg = 1
          else split2<F16>(S.rg[ig], S.rg[ig + 1], sg, h, l);
          GH[e] = h; GL[e] = l;
        }
        if (q < RJ / 8) {
          const int id = RJ * hh + 8 * q + 2 * e;
          if constexpr (SD != 0) h = S.rd[id] | (S.rd[id + 1] << 16);
          else split2<F16>(S.rd[id], S.rd[id + 1], sd, h, l);
          DH[e] = h; DL[e] = l;
        }
      }
      if (q < RJ / 8) {
        const int offd = wx3_off(ml, (rbase & 127) / 8 + q);
        *reinterpret_cast<u32x4*>(dbase + offd) = DH;
        if constexpr (PL == 2) *reinterpret_cast<u32x4*>(dbase + PLANE + offd) = DL;
      }
      if (q < RJG / 8 && (!KP || gact)) {
        const int offg = wx3_off(ml, (rbase_g & 127) / 8 + q);
        *reinterpret_cast<u32x4*>(gbase + offg) = GH;
        if constexpr (PL == 2) *reinterpret_cast<u32x4*>(gbase + PLANE + offg) = GL;
      }
    }
   }
  };

  f32x16 acc[RK][RN];
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int BMS = BMR * KH;              // positions per staging round
  const int nsteps = (mend > mbeg) ? (mend - mbeg + BMS - 1) / BMS : 0;
  // transposed-read addressing (T10): group g = lane >> 4 takes columns
  // 16 (g & 1) .. +15 of a 32-row block and positions 8 (g >> 1) + 0..3 / 4..7;
  // lane 4q + p of the group addresses position row q, columns 4p .. 4p + 3
  const int g = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
  auto frag = [&](const unsigned char* plane, int row0, int pos0) __attribute__((always_inline)) {
    const int c0 = (row0 + 16 * (g & 1)) >> 3;
    const int s0 = pos0 + 8 * (g >> 1) + gq;
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(plane + wx3_off(s0, c0 + (gp >> 1)) + 8 * (gp & 1)));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(plane + wx3_off(s0 + 4, c0 + (gp >> 1)) + 8 * (gp & 1)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int cur) __attribute__((always_inline)) {
    const unsigned char* base = sm[cur];
#pragma unroll
    for (int hs = 0; hs < 2 * KH; ++hs) {   // (half, 16-position k-substep)
      const int hh = hs >> 1, ks = hs & 1;
      if constexpr (KB > 1) {   // 128-row waves: one G row block's fragments live at a time
        bf16x8 gb[RN][PL];
#pragma unroll
        for (int p = 0; p < PL; ++p)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            gb[j][p] = frag(base + (DPL + 2 * (wnn >> 1) + p + hh) * PLANE, (wnn & 1) * TN + 32 * j, 16 * ks);
#pragma unroll
        for (int i = 0; i < RK; ++i) {
          const int krow = wk * TK + 32 * i;
          bf16x8 gi[PL];
#pragma unroll
          for (int p = 0; p < PL; ++p) gi[p] = frag(base + (2 * (krow >> 7) + p + hh) * PLANE, krow & 127, 16 * ks);
#pragma unroll
          for (int t = 0; t < TERMS; ++t)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = mfma_32x32x16<F16>(__builtin_bit_cast(u32x4, gi[t == 2 ? 1 : 0]),
                                             __builtin_bit_cast(u32x4, gb[j][t == 1 ? 1 : 0]), acc[i][j]);
        }
        continue;
      }
      bf16x8 ga[RK][PL], gb[RN][PL];
#pragma unroll
      for (int p = 0; p < PL; ++p) {
#pragma unroll
        for (int i = 0; i < RK; ++i)
          if (!KP || 32 * i < kvw) {
            const int krow = wk * TK + 32 * i;   // G block krow / 128
            ga[i][p] = frag(base + (2 * (krow >> 7) + p + hh) * PLANE, krow & 127, 16 * ks);
          }
#pragma unroll
        for (int j = 0; j < RN; ++j)
          gb[j][p] = frag(base + (DPL + 2 * (wnn >> 1) + p + hh) * PLANE, (wnn & 1) * TN + 32 * j, 16 * ks);
      }
#pragma unroll
      for (int t = 0; t < TERMS; ++t)
#pragma unroll
        for (int i = 0; i < RK; ++i)
          if (!KP || 32 * i < kvw)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = mfma_32x32x16<F16>(__builtin_bit_cast(u32x4, ga[i][t == 2 ? 1 : 0]),
                                             __builtin_bit_cast(u32x4, gb[j][t == 1 ? 1 : 0]), acc[i][j]);
    }
  };
  auto interleave = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int i = 0; i < 2 * TERMS * RK * RN * KH; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
      __builtin_amdgcn_sched_group_barrier(0x080, 2, 0);              // DS
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);              // global load
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);              // VALU
    }
  };
  if (nsteps > 0) {
    load_step(st0, mbeg);
    store_step(st0, 0);
  }
  int s = 0;
  if constexpr (KH > 1 || (KB > 1 && NB > 1)) {
    // one register staging set (prefetch distance one round = two 32-position steps,
    // as the two sets of the 32-position form): a round's loads are in flight during
    // the previous round's 16 MFMAs (256 x 128 tiles: two sets, 24 staged rows a thread)
    __syncthreads();
    for (; s + 1 < nsteps; s += 2) {
      load_step(st0, mbeg + (s + 1) * BMS);
      compute(0);
      store_step(st0, 1);
      interleave();
      __syncthreads();
      load_step(st0, mbeg + (s + 2) * BMS);
      compute(1);
      store_step(st0, 0);
      interleave();
      __syncthreads();
    }
  } else {
  if (nsteps > 1) load_step(st1, mbeg + BMS);
  __syncthreads();
  for (; s + 1 < nsteps; s += 2) {
    load_step(st0, mbeg + (s + 2) * BMS);
    compute(0);
    store_step(st1, 1);
    interleave();
    __syncthreads();
    load_step(st1, mbeg + (s + 3) * BMS);
    compute(1);
    store_step(st0, 0);
    interleave();
    __syncthreads();
  }
  }
  if (s < nsteps) compute(0);
  float* out = a.slab + (long long)split * a.Kp * a.Np;
  const int lk = lane >> 5, lc = lane & 31;
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = k0 + wk * TK + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const int n = n0 + wnn * TN + 32 * j + lc;
        out[(long long)k * a.Np + n] = F16 ? __builtin_ldexpf(acc[i][j][r], ush) : acc[i][j][r];
      }
  __syncthreads();   // the next tile restages sK and sm
  }
}

// ---------------------------------------------------------------------------
// Three-way split ("bf16x6"): x = h + m + l (each bf16, h = rne(x),
// m = rne(x - h), l = rne(x - h - m); both subtractions exact), 24 significant
// bits like fp32. Six MFMA terms keep every product of order >= 2^-16:
//   hh + hm + mh + hl + lh + mm   (dropped: ml, lm ~ 2^-24, ll ~ 2^-32)
// so the contraction is fp32-class (per-product error ~2^-23) at 6/16 of the
// fp32 MFMA cycles. Used for the forward pass, whose activation perturbation
// the ill-conditioned CBN parameter gradients amplify (tools/grad_modes.py).
// Tiles as gather_x3_kernel but BK = 16 per step (3 planes x 32-B rows).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void split3_bf16x2(float x0, float x1, unsigned& hi, unsigned& mid,
                                              unsigned& lo) {
  split_bf16x2(x0, x1, hi, mid);
  const float m0 = __builtin_bit_cast(float, mid << 16);
  const float m1 = __builtin_bit_cast(float, mid & 0xffff0000u);
  const float h0 = __builtin_bit_cast(float, hi << 16);
  const float h1 = __builtin_bit_cast(float, hi & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){(x0 - h0) - m0, (x1 - h1) - m1}, bf16x2));
}

constexpr int kX6BK = 16;
constexpr int kX6TileU4 = 3 * 128 * 2;   // u32x4 per (k-step, n-tile) weight image = 12 KB
// 32-B rows (2 chunks): chunk c of row r at c ^ ((r >> 3) & 1) -> ds_read_b128
// fragment reads conflict-free in every 16-lane group
__device__ __forceinline__ int x6_chunk(int row, int c) { return c ^ ((row >> 3) & 1); }

// Wt[(s * NT + t) * kX6TileU4 + (plane * 128 + n) * 2 + x6_chunk(n, c)]: element e of
// k = 16 s + 8 c + e, column 128 t + n. Also ktab.
__global__ void prep_class_x6_kernel(WeightView w, TapList taps, int Cg, int N, int Kp, int NT,
                                     int Hi, int Wi, int data_grad, int kblk, unsigned short* Wt,
                                     int4* ktab) {
  const int K = taps.n * Cg;
  const long long total = (long long)Kp * NT * 128;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(idx % Kp);
    const int n = (int)(idx / Kp);
    float v = 0.f;
    if (k < K && n < N) {
      int t, c;
      split_k(k, Cg, taps.n, kblk, t, c);
      const int ci = data_grad ? n : c, co = data_grad ? c : n;
      v = kernel_value(w, ci, co, taps.ti[t], taps.tj[t]);
    }
    const float h = (float)(__bf16)v;
    const float mv = (float)(__bf16)(v - h);
    const unsigned short hb = bf16_bits(v), mb = bf16_bits(v - h), lb = bf16_bits((v - h) - mv);
    const int s = k >> 4, kc = (k >> 3) & 1, e = k & 7;
    const int tn = n >> 7, nl = n & 127;
    const long long base = ((long long)s * NT + tn) * kX6TileU4 * 8;
    const long long off = ((long long)nl * 2 + x6_chunk(nl, kc)) * 8 + e;
    Wt[base + off] = hb;
    Wt[base + 128 * 2 * 8 + off] = mb;
    Wt[base + 2 * 128 * 2 * 8 + off] = lb;
    if (n == 0) {
      int4 q;
      q.w = 0;
      if (k < K) {
        int t, c;
        split_k(k, Cg, taps.n, kblk, t, c);
        q.x = (int)((long long)c * Hi * Wi + (long long)taps.offh[t] * Wi + taps.offw[t]);
        q.y = taps.offh[t];
        q.z = taps.offw[t];
        q.w = c;
      } else {
        q.x = 0; q.y = kInvalidOff; q.z = 0;
      }
      ktab[k] = q;
    }
  }
}

// JG: the gathered tensor is the decoder skip join (as gather_x3_kernel JM = 1).
// NW: 128-column weight tiles per workgroup (as gather_x3_kernel); with NW = 2
// a thread gathers 4 k per step and writes half-chunks (ds_write_b64).
template <bool TU, bool JG = false, int NW = 1>
__global__ void __launch_bounds__(kThreads * NW, NW == 1 ? 2 : 1)
gather_x6_kernel(const GatherArgs a) {
  static_assert(!JG || TU, "the joined gather runs on the tap-uniform path");
  static_assert(NW == 1 || NW == 2, "128 or 256 columns per workgroup");
  constexpr int THR = kThreads * NW;
  constexpr int BN = kX3BN * NW, BM = kX3BM, WM = 2, TN = 64, TM = 64, RN = 2, RM = 2;
  constexpr int BK = kX6BK, AJ = 8 / NW;          // gathered k per thread per step
  __shared__ __attribute__((aligned(16))) u32x4 sA[2][3 * BM * 2];
  __shared__ __attribute__((aligned(16))) u32x4 sW[2][3 * BN * 2];   // [t][plane][128 rows][2]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int NT = gridDim.y;                       // workgroup column tiles (BN wide)
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const long long HiWi = (long long)a.Hi * a.Wi;

  const int am = tid % BM;
  const int akr = __builtin_amdgcn_readfirstlane(tid / BM);   // 0 .. 2 NW - 1 (wave-uniform)
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
  struct Stage { float ra[AJ]; u32x4 rw[3]; };
  Stage s0, s1;
  using se::uniform_ptr;
  const int b0 = m0 / (a.Qh * a.Qw);
  const int cpb = JG ? 2 * a.jh : a.Cg;           // channels per batch item of X
  const long long H2W2 = (long long)a.H2 * a.W2;
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.X + (long long)b0 * cpb * HiWi), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rx2 = rx;
  if constexpr (JG)
    rx2 = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(a.X2 + (long long)b0 * cpb * H2W2), (short)0,
                                            0x7FFFFFFF, 0x00020000);
  const u32x4* wt = reinterpret_cast<const u32x4*>(a.Wp) + (long long)nt * NW * kX6TileU4 + tid;
  int xoff = 0, xoff2 = 0;
  if constexpr (TU) {
    if (mval) {
      const int b = m / (a.Qh * a.Qw);
      xoff = (int)(((long long)(b - b0) * cpb * HiWi + (long long)hb * a.Wi + wb) * 4);
      if constexpr (JG) xoff2 = (int)(((long long)(b - b0) * cpb * H2W2 + (long long)hb * a.W2 + wb) * 4);
    }
  }
  auto load_tile = [&](Stage& st, int k0) __attribute__((always_inline)) {
    if constexpr (TU) {
      const int4 e0 = a.ktab[k0];                 // the step's tap and first channel (uniform)
      int c0 = e0.w;
      const int hi = hb + e0.y, wi = wb + e0.z;
      bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      int vo = xoff + (e0.y * a.Wi + e0.z) * 4, cs = (int)(HiWi * 4);
      __amdgpu_buffer_rsrc_t r = rx;
      if constexpr (JG) {                         // a K-step lies in one join chunk
        const int q = c0 / a.jh;                  // chunk order as gather_x3_kernel
        const bool from_x = a.jcat ? q < 2 : (q & 1) == 0;
        c0 = (a.jcat ? (q & 1) : (q >> 1)) * a.jh + (c0 - q * a.jh);
        ok &= !from_x | ((hi < a.H2) & (wi < a.W2));   // F.pad rows / columns of x read 0
        vo = from_x ? xoff2 + (e0.y * a.W2 + e0.z) * 4 : vo;
        cs = from_x ? (int)(H2W2 * 4) : cs;
        r = from_x ? rx2 : rx;
      }
      vo = ok ? vo : (int)0x80000000;
      c0 += AJ * akr;
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        st.ra[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, (c0 + j) * cs, 0));
    } else {
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int4 e = a.ktab[k0 + AJ * akr + j];
        const int hi = hb + e.y, wi = wb + e.z;
        const bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
        st.ra[j] = *(ok ? a.X + xbase + e.x : a.zero);
      }
    }
    const u32x4* src = wt + (long long)(k0 / BK) * NT * NW * kX6TileU4;
#pragma unroll
    for (int j = 0; j < 3; ++j) st.rw[j] = src[THR * j];
  };
  const int wchunk = x6_chunk(am, AJ == 8 ? akr : akr >> 1);
  auto store_tile = [&](const Stage& st, int buf) __attribute__((always_inline)) {
    if constexpr (AJ == 8) {
      u32x4 H, M, L;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned h, mm, l;
        split3_bf16x2(st.ra[2 * e], st.ra[2 * e + 1], h, mm, l);
        H[e] = h; M[e] = mm; L[e] = l;
      }
      sA[buf][am * 2 + wchunk] = H;
      sA[buf][BM * 2 + am * 2 + wchunk] = M;
      sA[buf][2 * BM * 2 + am * 2 + wchunk] = L;
    } else {                                      // half a chunk: k 4 (akr & 1) .. + 3
      typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
      u32x2v H, M, L;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        unsigned h, mm, l;
        split3_bf16x2(st.ra[2 * e], st.ra[2 * e + 1], h, mm, l);
        H[e] = h; M[e] = mm; L[e] = l;
      }
      const int half = akr & 1;
      reinterpret_cast<u32x2v*>(&sA[buf][am * 2 + wchunk])[half] = H;
      reinterpret_cast<u32x2v*>(&sA[buf][BM * 2 + am * 2 + wchunk])[half] = M;
      reinterpret_cast<u32x2v*>(&sA[buf][2 * BM * 2 + am * 2 + wchunk])[half] = L;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) sW[buf][tid + THR * j] = st.rw[j];
  };

  f32x16 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lh = lane >> 5, lr = lane & 31;
  const int fc = x6_chunk(lr, lh);
  auto compute = [&](int cur) __attribute__((always_inline)) {
    u32x4 wf[RN][3], af[RM][3];   // [block][plane]
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < RN; ++i) {
        const int n = wn * TN + 32 * i;           // block's first column (uniform)
        wf[i][p] = sW[cur][(((n >> 7) * 3 + p) * 128 + (n & 127) + lr) * 2 + fc];
      }
#pragma unroll
      for (int j = 0; j < RM; ++j) af[j][p] = sA[cur][(p * BM + wm * TM + 32 * j + lr) * 2 + fc];
    }
    // terms (weight plane, activation plane), small terms first
    constexpr int TA[6] = {1, 2, 0, 1, 0, 0};
    constexpr int TB[6] = {1, 0, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int i = 0; i < RN; ++i)
#pragma unroll
        for (int j = 0; j < RM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              __builtin_bit_cast(bf16x8, wf[i][TA[t]]), __builtin_bit_cast(bf16x8, af[j][TB[t]]),
              acc[i][j], 0, 0, 0);
  };
  auto interleave = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                // MFMA
      if (i < 14) __builtin_amdgcn_sched_group_barrier(0x080, 1, 0);    // DS
      if (i < AJ + 3) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // global load
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);                // VALU
    }
  };

  const int nk = a.Kp / BK;
  load_tile(s0, 0);
  store_tile(s0, 0);
  if (nk > 1) load_tile(s1, BK);
  __syncthreads();
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    load_tile(s0, min(kt + 2, nk - 1) * BK);
    compute(0);
    store_tile(s1, 1);
    interleave();
    __syncthreads();
    load_tile(s1, min(kt + 3, nk - 1) * BK);
    compute(1);
    store_tile(s0, 0);
    interleave();
    __syncthreads();
  }
  if (kt < nk) compute(0);

  __syncthreads();
  float* sBias = reinterpret_cast<float*>(&sW[0][0]);
  for (int i = tid; i < BN; i += THR) {
    const int n = n0 + i;
    sBias[i] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
  }
  __syncthreads();
  const long long HoWo = (long long)a.Ho * a.Wo;
  const bool full_n = n0 + BN <= a.N;
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const int mm = m0 + wm * TM + 32 * j + lr;
    if (mm >= a.M) continue;
    const int qhw = a.Qh * a.Qw;
    const int b = mm / qhw, r = mm - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    const int nl0 = wn * TN + 4 * lh;
    float* yb = a.Y + (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo +
                (a.pw + a.Sw * qw) + (long long)(n0 + nl0) * HoWo;
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        const int nl = 32 * i + (r2 & 3) + 8 * (r2 >> 2);
        if (full_n || n0 + nl0 + nl < a.N) yb[(long long)nl * HoWo] = acc[i][j][r2] + sBias[nl0 + nl];
      }
  }
}
