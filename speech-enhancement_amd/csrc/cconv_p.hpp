// Pipelined split-fp16 gather GEMM (SE_MATH_F16X3, tap-uniform): the forward and
// data-grad of the fused complex (transposed) conv, included by cconv.hip after
// cconv_x3.hpp (same GatherArgs, weight image and epilogue conventions).
//
// gather_x3_kernel reads ALL fragments of a K-step right after the step's barrier and
// only then issues its MFMAs, so every wave of the CU starts a step with an LDS burst
// (8 waves x 16 ds_read_b128) while the matrix cores idle: the round-3/4 counters put
// the MFMA pipe at ~0.5 busy behind s_waitcnt / barrier stalls. Here:
//  * the tile is 256 positions (m) x 64 NWN outputs (n), 2 NWN waves of 128 m x 64 n
//    (4 x 2 accumulator blocks of v_mfma_f32_32x32x16_f16): a third fewer LDS
//    fragment bytes per MFMA than 64 x 64 per wave;
//  * K advances in stages of 16 in a 3-slot LDS ring. While the MFMAs of stage s run,
//    the same wave reads the fragments of stage s + 1 (block by block, into the
//    registers the finished block frees) and stores stage s + 2's operands (gathered
//    and split two stages earlier) into the third slot; one barrier per stage;
//  * the gathered activations are loaded two stages ahead (two register sets; NWN = 2,
//    whose threads stage twice the values, one set one stage ahead, two workgroups per
//    CU covering each other's latency), the weights come from the same pre-split image
//    as gather_x3_kernel.
// Per accumulator the MFMA sequence (k16 blocks in order, terms hi*hi, hi*lo, lo*hi)
// equals gather_x3_kernel's, and the split and image are the same, so the results are
// bit-identical to it (tests/test_gpu_conv_x3.py checks this through a variant build).
//
// NWN = 4: 256 x 256 tiles, 512 threads, 96 KB LDS, one workgroup per CU (N = 256:
//          the joined decoder data-grad). NWN = 2: 256 x 128, 256 threads, 72 KB, two
//          per CU (N = 128: the encoder passes and the joined decoder forward).
// JM: decoder skip join (as gather_x3_kernel): 1 joined input, 2 joined output.

constexpr int kPBM = 256;    // positions per tile
constexpr int kPBK = 16;     // k per stage
constexpr int kPSlots = 3;   // LDS ring depth

template <int JM, int NWN>
__global__ void __launch_bounds__(128 * NWN, NWN == 4 ? 1 : 2)
gather_p_kernel(const GatherArgs a) {
  static_assert(NWN == 2 || NWN == 4, "128 or 256 output columns per tile");
  constexpr int THR = 128 * NWN;
  constexpr int BN = 64 * NWN;
  constexpr int WPL = BN * 32, XPL = kPBM * 32;    // bytes of one plane (rows x 2 chunks of 16 B)
  constexpr int XOFF = 2 * WPL;                    // X planes after the two W planes of a slot
  constexpr int SLOT = 2 * WPL + 2 * XPL;
  constexpr int XJ = kPBM * kPBK / THR;            // gathered values per thread per stage (8 or 16)
  __shared__ __attribute__((aligned(16))) unsigned char sm[kPSlots * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % NWN, wm = wave / NWN;
  const int NT = gridDim.y;
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * kPBM, n0 = nt * BN;
  const long long HiWi = (long long)a.Hi * a.Wi;
  const int nk = a.Kp / kPBK;

  // ---- activation gather: thread -> position xm of the tile, k values xk0 .. xk0 + XJ - 1
  const int xm = tid & (kPBM - 1);
  const int xk0 = XJ == 16 ? 0 : 8 * (tid >> 8);
  const int m = m0 + xm;
  const bool mval = m < a.M;
  int hb = 0, wb = 0, xoff = 0, xoff2 = 0;
  const int qhw = a.Qh * a.Qw;
  const int b0 = m0 / qhw;
  const int cpb = JM == 1 ? 2 * a.jh : a.Cg;       // channels per batch item of X
  const long long H2W2 = (long long)a.H2 * a.W2;
  if (mval) {
    const int b = m / qhw, r = m - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    hb = qh * a.sh;
    wb = qw * a.sw;
    xoff = (int)(((long long)(b - b0) * cpb * HiWi + (long long)hb * a.Wi + wb) * 4);
    if constexpr (JM == 1) xoff2 = (int)(((long long)(b - b0) * cpb * H2W2 + (long long)hb * a.W2 + wb) * 4);
  }
  using se::uniform_ptr;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(a.X + (long long)b0 * cpb * HiWi), (short)0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rx2 = rx;
  if constexpr (JM == 1)
    rx2 = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(a.X2 + (long long)b0 * cpb * H2W2), (short)0,
                                            0x7FFFFFFF, 0x00020000);
  const int ea = amax_exp(a.amax_a);
  const float sa = pow2f(kF16Top - ea);
  const int ush = ea + amax_exp(a.amax_w) - 2 * kF16Top;

  // ---- weights: thread -> image row wrow (of BN), chunk wcl of the stage's two, both planes
  const int wrow = tid >> 1, wcl = tid & 1;
  const int wng = n0 + wrow;                       // global weight column
  const int NT128 = a.ldw >> 7;                    // 128-column tiles of the image
  const u32x4* wimg = reinterpret_cast<const u32x4*>(a.Wp);
  const int wrow128 = wng & 127;
  const int wbase = (wng >> 7) * kX3TileU4 + wrow128 * 4;

  struct Stg { float x[XJ]; u32x4 w[2]; };
  auto load = [&](Stg& g, int t) __attribute__((always_inline)) {
    t = min(t, nk - 1);                            // past the end: a harmless reload
    const int k0 = kPBK * t;
    const int4 e0 = a.ktab[k0];                    // the stage's tap and first channel (uniform)
    int c0 = e0.w;
    const int hi = hb + e0.y, wi = wb + e0.z;
    bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
    int vo = xoff + (e0.y * a.Wi + e0.z) * 4, cs = (int)(HiWi * 4);
    __amdgpu_buffer_rsrc_t r = rx;
    if constexpr (JM == 1) {                       // a stage lies in one join chunk (jh % 16 == 0)
      const int q = c0 / a.jh;
      const bool from_x = a.jcat ? q < 2 : (q & 1) == 0;
      c0 = (a.jcat ? (q & 1) : (q >> 1)) * a.jh + (c0 - q * a.jh);
      ok &= !from_x | ((hi < a.H2) & (wi < a.W2));
      vo = from_x ? xoff2 + (e0.y * a.W2 + e0.z) * 4 : vo;
      cs = from_x ? (int)(H2W2 * 4) : cs;
      r = from_x ? rx2 : rx;
    }
    vo = ok ? vo : (int)0x80000000;
    c0 += xk0;
#pragma unroll
    for (int j = 0; j < XJ; ++j) g.x[j] = bload<0>(r, vo, (c0 + j) * cs);
    // 32-k image step t / 2, chunk 2 (t & 1) + wcl of row wrow128, swizzled as prep_class_x3_kernel
    const int c = 2 * (t & 1) + wcl;
    const u32x4* src = wimg + (long long)(t >> 1) * NT128 * kX3TileU4 + wbase + x3_chunk(wrow128, c);
    g.w[0] = src[0];
    g.w[1] = src[128 * 4];
  };
  // LDS images: [plane][row][2 chunks], chunk stored at c ^ (bit 4 of the row)
  const int xst = (xm * 32) + 0;                   // row base of this thread's position
  auto store = [&](const Stg& g, int slot) __attribute__((always_inline)) {
    unsigned char* b = sm + slot * SLOT;
    const int wofs = wrow * 32 + ((wcl ^ ((wrow >> 4) & 1)) << 4);
    *reinterpret_cast<u32x4*>(b + wofs) = g.w[0];
    *reinterpret_cast<u32x4*>(b + WPL + wofs) = g.w[1];
#pragma unroll
    for (int q = 0; q < XJ / 8; ++q) {
      u32x4 H, L;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned h, l;
        split2<true>(g.x[8 * q + 2 * e], g.x[8 * q + 2 * e + 1], sa, h, l);
        H[e] = h;
        L[e] = l;
      }
      const int ch = (xk0 >> 3) + q;               // chunk of the stage's 16 k
      const int xofs = XOFF + xst + ((ch ^ ((xm >> 4) & 1)) << 4);
      *reinterpret_cast<u32x4*>(b + xofs) = H;
      *reinterpret_cast<u32x4*>(b + XPL + xofs) = L;
    }
  };
  // fragments: W rows wn * 64 + 32 i + lr, X rows wm * 128 + 32 j + lr, chunk lh
  const int lr = lane & 31, lh = lane >> 5;
  const int fc = (lh ^ ((lr >> 4) & 1)) << 4;
  const int fw = (wn * 64 + lr) * 32 + fc, fx = XOFF + (wm * 128 + lr) * 32 + fc;
  struct Frags { u32x4 w[4], x[8]; };              // w[2 i + plane], x[2 j + plane]
  auto read_w = [&](Frags& F, int slot) __attribute__((always_inline)) {
    const unsigned char* b = sm + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) F.w[2 * i + p] = *reinterpret_cast<const u32x4*>(b + fw + p * WPL + 32 * 32 * i);
  };
  auto read_x = [&](Frags& F, int slot, int j) __attribute__((always_inline)) {
    const unsigned char* b = sm + slot * SLOT;
#pragma unroll
    for (int p = 0; p < 2; ++p) F.x[2 * j + p] = *reinterpret_cast<const u32x4*>(b + fx + p * XPL + 32 * 32 * j);
  };
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // the MFMAs of one stage block by block (X block j outer: hi*hi, hi*lo, lo*hi of both W
  // blocks), each X block's registers refilled with the next stage's fragments after it
  auto compute_read = [&](const Frags& F, Frags& G, int slot_next) __attribute__((always_inline)) {
    read_w(G, slot_next);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = mfma_32x32x16<true>(F.w[2 * i + (t == 2)], F.x[2 * j + (t == 1)], acc[i][j]);
      read_x(G, slot_next, j);
    }
  };

  Frags F0, F1;
  // iteration pair (s, s + 1): stage s's MFMAs use fragments read from slot s % 3 (in F0),
  // stage s + 1's fragments come from slot (s + 1) % 3, stage s + 2 is stored into
  // (s + 2) % 3; past the last stage the loads repeat it and the stores fill slots whose
  // contents are never used
  int slot = 0;
  if constexpr (NWN == 4) {   // two staging sets: loads two stages ahead
    Stg g0, g1;
    load(g0, 0);
    load(g1, 1);
    store(g0, 0);
    load(g0, 2);
    store(g1, 1);
    load(g1, 3);
    __syncthreads();
    read_w(F0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) read_x(F0, 0, j);
    for (int s = 0; s < nk; s += 2) {
      const int s1 = slot == 2 ? 0 : slot + 1, s2 = s1 == 2 ? 0 : s1 + 1;
      compute_read(F0, F1, s1);
      store(g0, s2);
      load(g0, s + 4);
      __syncthreads();
      compute_read(F1, F0, s2);
      store(g1, slot);                              // slot s % 3 == (s + 3) % 3
      load(g1, s + 5);
      __syncthreads();
      slot = s2;
    }
  } else {                    // one staging set: loads one stage ahead
    Stg g;
    load(g, 0);
    store(g, 0);
    load(g, 1);
    store(g, 1);
    load(g, 2);
    __syncthreads();
    read_w(F0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) read_x(F0, 0, j);
    for (int s = 0; s < nk; s += 2) {
      const int s1 = slot == 2 ? 0 : slot + 1, s2 = s1 == 2 ? 0 : s1 + 1;
      compute_read(F0, F1, s1);
      store(g, s2);
      load(g, s + 3);
      __syncthreads();
      compute_read(F1, F0, s2);
      store(g, slot);
      load(g, s + 4);
      __syncthreads();
      slot = s2;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], ush);

  // ---- epilogue (as gather_x3_kernel): block (i, j) element r is column (m) 32 j + lr
  // and row (n) 32 i + 4 lh + (r & 3) + 8 (r >> 2) of the wave tile
  const long long HoWo = (long long)a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int mm = m0 + wm * 128 + 32 * j + lr;
    if (mm >= a.M) continue;
    const int b = mm / qhw, r = mm - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    if constexpr (JM == 2) {
      const int oh = a.ph + a.Sh * qh, ow = a.pw + a.Sw * qw;
      const long long P2 = (long long)a.YH2 * a.YW2;
      const int ycpb = 2 * a.yjh;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int nb = n0 + wn * 64 + 32 * i;      // block's first channel (wave-uniform)
        const int q = nb / a.yjh;
        const int cb = (a.jcat ? (q & 1) : (q >> 1)) * a.yjh + (nb - q * a.yjh) + 4 * lh;
        const bool to_x = a.jcat ? q < 2 : (q & 1) == 0;
        if (to_x && (oh >= a.YH2 || ow >= a.YW2)) continue;
        const long long pl = to_x ? P2 : HoWo;
        float* yp = to_x ? a.Y2 + ((long long)b * ycpb + cb) * P2 + (long long)oh * a.YW2 + ow
                         : a.Y + ((long long)b * ycpb + cb) * HoWo + (long long)oh * a.Wo + ow;
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) yp[(long long)((r2 & 3) + 8 * (r2 >> 2)) * pl] = acc[i][j][r2];
      }
    } else {
      const int nl0 = wn * 64 + 4 * lh;
      const long long yb = (long long)b * a.N * HoWo + (long long)(a.ph + a.Sh * qh) * a.Wo +
                           (a.pw + a.Sw * qw) + (long long)(n0 + nl0) * HoWo;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) {
          const int nl = 32 * i + (r2 & 3) + 8 * (r2 >> 2);
          const int n = n0 + nl0 + nl;
          if (n < a.N) a.Y[yb + (long long)nl * HoWo] = acc[i][j][r2] + (a.bias ? a.bias[n] : 0.f);
        }
    }
  }
}
