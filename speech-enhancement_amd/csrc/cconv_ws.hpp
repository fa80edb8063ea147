// Warp-specialised form of the scaled split-fp16 gather GEMM (included by cconv.hip after
// cconv_x3.hpp, inside its anonymous namespace). Same contraction, operand images, tile
// (256 n x 128 m, eight 64 x 64 MFMA waves) and epilogue as
// gather_x3_kernel<true, 3, JM, 2, true, 0>; the schedule differs:
//
//   - 4 loader waves gather + split the operand tiles of each K-step into a 3-deep LDS
//     ring (144 KB) and publish a slot with an LDS counter (full[slot] += 1 per wave);
//   - 8 MFMA waves wait on full[slot], read their fragments, hand the slot back
//     (empty[slot] += 1 per wave) and issue the step's 24 MFMAs;
//
// so no wave ever waits at a workgroup barrier inside the K loop: an MFMA wave waits only
// for the slot it needs, a loader wave only for the slot it refills (the round-4 / round-5
// ask). Counters only grow: use u of slot s is full when full[s] = 4 (u + 1) and free
// again when empty[s] = 8 (u + 1). Every wait is bounded (kWsSpinLimit polls of
// s_sleep 1, ~0.5 s): a wave that runs out leaves its loop, so a broken handshake
// gives wrong numbers (caught by the parity tests), never a hung GPU.
//
// SEHIP_X3_WS=1 selects it for the 256-column f16x3 passes on fp32 storage; the
// default stays gather_x3_kernel until it measures faster (profiles/ab/r6_x3_ws_*).

constexpr int kWsSlots = 3, kWsLoaders = 4, kWsMaxSteps = 512;
// MFMA waves: 8 of 64 x 64, or (V & 4, "big") 4 of 128 x 64 whose fragment reads are a
// quarter fewer LDS bytes per MFMA, software-pipelined by k-substep
template <int V> constexpr int ws_mma_waves() { return (V & 4) ? 4 : 8; }
template <int V> constexpr int ws_threads() { return 64 * (kWsLoaders + ws_mma_waves<V>()); }
constexpr int kWsSpinLimit = 1 << 23;

// The handshake orders LDS only. A workgroup-scope acquire / release on a generic
// pointer would also wait for the loader waves' outstanding global loads (vmcnt(0)),
// i.e. drain the prefetch every K-step; so the counters are relaxed atomics behind
// compiler-only fences, and the release waits for the LDS counter alone (a wave's LDS
// operations complete in order; the flag load is consumed by the loop branch before
// any later slot read issues).
template <bool SLEEP = true>
__device__ __forceinline__ void ws_wait_geq(int* flag, int target) {
  int spins = 0;
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target &&
         ++spins < (SLEEP ? kWsSpinLimit : 16 * kWsSpinLimit))
    if (SLEEP) __builtin_amdgcn_s_sleep(1);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ void ws_signal(int* flag, int lane) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS reads / writes of the slot are done
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (lane == 0) __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// V (A/B variants, SEHIP_X3_WS = 1 + V): bit 0 = an MFMA wave hands its slot back after
// the first k-substep's MFMAs are issued (the second substep's fragment reads overlap
// them); bit 1 = poll without s_sleep
template <int JM, int V = 0>
__global__ void __launch_bounds__(ws_threads<V>(), 1) gather_ws_kernel(const GatherArgs a) {
  constexpr bool SLEEP = !(V & 2), SPLIT = V & 1, BIG = V & 4;
  constexpr int kWsMma = ws_mma_waves<V>();
  constexpr int NW = 2, BN = kX3BN * NW, BM = kX3BM, WM = 2, TM = 64, RM = 2, PL = 2;
  constexpr int RN = BIG ? 4 : 2, TN = 32 * RN;
  constexpr int VT = kThreads * NW;          // the 512 staging threads of gather_x3_kernel<.., NW = 2>
  constexpr int AJ = 16 / NW;                // gathered k per staging thread per K-step
  __shared__ __attribute__((aligned(16))) u32x4 sA[kWsSlots][2 * BM * 4];
  __shared__ __attribute__((aligned(16))) u32x4 sW[kWsSlots][2 * BN * 4];
  __shared__ int full[kWsSlots], empty[kWsSlots];
  // the K-steps' tap-table entries, staged once: in the K loop a global (vector) load of
  // the entry would queue behind the previous step's gathers, and waiting for it would
  // drain them (the host checks nk <= kWsMaxSteps)
  __shared__ int4 sK[kWsMaxSteps];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform role branch, scalar tap-table loads
  if (tid < kWsSlots) { full[tid] = 0; empty[tid] = 0; }
  for (int k = tid; k < a.Kp / kBK; k += blockDim.x) sK[k] = a.ktab[k * kBK];
  __syncthreads();   // the only workgroup barrier

  const int NT = gridDim.y;
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const long long HiWi = (long long)a.Hi * a.Wi;
  const int nk = a.Kp / kBK;

  if (wave >= kWsMma) {
    // ---------------- loader waves: staging threads pt and pt + 256 of the 512-thread map
    const int pt = tid - 64 * kWsMma;                          // 0 .. 255
    const int am = pt % BM;                                    // both share the column
    const int akr0 = __builtin_amdgcn_readfirstlane(pt / BM);  // 0 / 1; the second is + 2
    const int m = m0 + am;
    const bool mval = m < a.M;
    int hb = 0, wb = 0, xoff = 0, xoff2 = 0;
    const int b0 = m0 / (a.Qh * a.Qw);
    const int cpb = JM == 1 ? 2 * a.jh : a.Cg;
    const long long H2W2 = (long long)a.H2 * a.W2;
    if (mval) {
      const int qhw = a.Qh * a.Qw;
      const int b = m / qhw, r = m - b * qhw;
      const int qh = r / a.Qw, qw = r - qh * a.Qw;
      hb = qh * a.sh;
      wb = qw * a.sw;
      xoff = (int)(((long long)(b - b0) * cpb * HiWi + (long long)hb * a.Wi + wb) * 4);
      if constexpr (JM == 1) xoff2 = (int)(((long long)(b - b0) * cpb * H2W2 + (long long)hb * a.W2 + wb) * 4);
    }
    const int ea = amax_exp(a.amax_a);
    const float sa = pow2f(kF16Top - ea);
    using se::uniform_ptr;
    __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr((const char*)a.X + (long long)b0 * cpb * HiWi * 4), (short)0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rx2 = rx;
    if constexpr (JM == 1)
      rx2 = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr((const char*)a.X2 + (long long)b0 * cpb * H2W2 * 4),
                                              (short)0, 0x7FFFFFFF, 0x00020000);
    const u32x4* wt = reinterpret_cast<const u32x4*>(a.Wp) + (long long)nt * NW * kX3TileU4;
    struct Stage { float ra[2 * AJ]; u32x4 rw[2 * 2 * PL]; };
    constexpr int S = BIG ? 4 : 2;   // register stages: loads run S - 1 K-steps ahead
    Stage st[S];
    auto load = [&](Stage& sg, int kt) __attribute__((always_inline)) {
      const int4 e0 = sK[kt];
      int c0 = e0.w;
      const int hi = hb + e0.y, wi = wb + e0.z;
      bool ok = mval & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      int vo = xoff + (e0.y * a.Wi + e0.z) * 4, cs = (int)(HiWi * 4);
      __amdgpu_buffer_rsrc_t r = rx;
      if constexpr (JM == 1) {
        const int q = c0 / a.jh;
        const bool from_x = a.jcat ? q < 2 : (q & 1) == 0;
        c0 = (a.jcat ? (q & 1) : (q >> 1)) * a.jh + (c0 - q * a.jh);
        ok &= !from_x | ((hi < a.H2) & (wi < a.W2));
        vo = from_x ? xoff2 + (e0.y * a.W2 + e0.z) * 4 : vo;
        cs = from_x ? (int)(H2W2 * 4) : cs;
        r = from_x ? rx2 : rx;
      }
      vo = ok ? vo : (int)0x80000000;
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int j = 0; j < AJ; ++j) sg.ra[AJ * v + j] = bload<0>(r, vo, (c0 + AJ * (akr0 + 2 * v) + j) * cs);
      const u32x4* src = wt + (long long)kt * NT * NW * kX3TileU4;
#pragma unroll
      for (int q = 0; q < 2 * 2 * PL; ++q) sg.rw[q] = src[pt + (VT / 2) * q];
    };
    const int swz = x3_swz(am);
    auto put = [&](const Stage& sg, int kt) __attribute__((always_inline)) {
      const int slot = kt % kWsSlots, use = kt / kWsSlots;
      ws_wait_geq<SLEEP>(&empty[slot], kWsMma * use);
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        u32x4 H, L;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned h, l;
          split2<true>(sg.ra[AJ * v + 2 * e], sg.ra[AJ * v + 2 * e + 1], sa, h, l);
          H[e] = h;
          L[e] = l;
        }
        const int c = (akr0 + 2 * v) ^ swz;
        sA[slot][am * 4 + c] = H;
        sA[slot][BM * 4 + am * 4 + c] = L;
      }
#pragma unroll
      for (int q = 0; q < 2 * 2 * PL; ++q) sW[slot][pt + (VT / 2) * q] = sg.rw[q];
      ws_signal(&full[slot], lane);
    };
    // unconditional (clamped) loads: with a load under a branch the compiler's wait
    // counting gives up and drains every load before each slot write
#pragma unroll
    for (int p = 0; p < S - 1; ++p) load(st[p], min(p, nk - 1));
    for (int kt = 0; kt < nk; kt += S) {
#pragma unroll
      for (int u = 0; u < S; ++u) {
        if (kt + u >= nk) break;
        load(st[(u + S - 1) % S], min(kt + u + S - 1, nk - 1));
        put(st[u], kt + u);
      }
    }
    return;
  }

  // ---------------- MFMA waves (the wave map of gather_x3_kernel<.., NW = 2>)
  const int wn = wave / WM, wm = wave % WM;
  const int ush = amax_exp(a.amax_a) + amax_exp(a.amax_w) - 2 * kF16Top;
  f32x16 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int lh = lane >> 5, lr = lane & 31;
  const int fsw = x3_swz(lr);
  // fragments of k-substep kk of a slot
  auto frags = [&](int slot, int kk, u32x4 (&wf)[RN][PL], u32x4 (&af)[RM][PL]) __attribute__((always_inline)) {
    const int c = (2 * kk + lh) ^ fsw;
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int n = wn * TN + 32 * i;
#pragma unroll
      for (int p = 0; p < PL; ++p) wf[i][p] = sW[slot][(((n >> 7) * PL + p) * 128 + (n & 127) + lr) * 4 + c];
    }
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int p = 0; p < PL; ++p) af[j][p] = sA[slot][(p * BM + wm * TM + 32 * j + lr) * 4 + c];
  };
  auto mma = [&](const u32x4 (&wf)[RN][PL], const u32x4 (&af)[RM][PL]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < RN; ++i)
#pragma unroll
        for (int j = 0; j < RM; ++j)
          acc[i][j] = mfma_32x32x16<true>(wf[i][t == 2 ? 1 : 0], af[j][t == 1 ? 1 : 0], acc[i][j]);
  };
  if constexpr (BIG) {
    // substep 1's reads overlap substep 0's MFMAs, the next step's substep-0 reads
    // overlap substep 1's
    u32x4 w0[RN][PL], a0[RM][PL], w1[RN][PL], a1[RM][PL];
    ws_wait_geq<SLEEP>(&full[0], kWsLoaders);
    frags(0, 0, w0, a0);
    for (int kt = 0; kt < nk; ++kt) {
      const int slot = kt % kWsSlots;
      frags(slot, 1, w1, a1);
      mma(w0, a0);
      ws_signal(&empty[slot], lane);
      if (kt + 1 < nk) {
        const int nx = (kt + 1) % kWsSlots;
        ws_wait_geq<SLEEP>(&full[nx], kWsLoaders * ((kt + 1) / kWsSlots + 1));
        frags(nx, 0, w0, a0);
      }
      mma(w1, a1);
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      const int slot = kt % kWsSlots, use = kt / kWsSlots;
      ws_wait_geq<SLEEP>(&full[slot], kWsLoaders * (use + 1));
      u32x4 wf[2][RN][PL], af[2][RM][PL];
      frags(slot, 0, wf[0], af[0]);
      frags(slot, 1, wf[1], af[1]);
      if (!SPLIT) ws_signal(&empty[slot], lane);
      mma(wf[0], af[0]);
      if (SPLIT) ws_signal(&empty[slot], lane);
      mma(wf[1], af[1]);
    }
  }
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], ush);

  // epilogue of gather_x3_kernel (the bias read from global: no barrier after the split)
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
    if constexpr (JM == 2) {
      const int oh = a.ph + a.Sh * qh, ow = a.pw + a.Sw * qw;
      const long long P2 = (long long)a.YH2 * a.YW2;
      const int cpb = 2 * a.yjh;
#pragma unroll
      for (int i = 0; i < RN; ++i) {
        const int nb = n0 + wn * TN + 32 * i;
        const int q = nb / a.yjh;
        const int cb = (a.jcat ? (q & 1) : (q >> 1)) * a.yjh + (nb - q * a.yjh) + 4 * lh;
        const bool to_x = a.jcat ? q < 2 : (q & 1) == 0;
        if (to_x && (oh >= a.YH2 || ow >= a.YW2)) continue;
        const long long pl = to_x ? P2 : HoWo;
        const long long yo = to_x ? ((long long)b * cpb + cb) * P2 + (long long)oh * a.YW2 + ow
                                  : ((long long)b * cpb + cb) * HoWo + (long long)oh * a.Wo + ow;
        float* yb = to_x ? a.Y2 : a.Y;
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) yb[yo + (long long)((r2 & 3) + 8 * (r2 >> 2)) * pl] = acc[i][j][r2];
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
        const int n = n0 + nl0 + nl;
        if (full_n || n < a.N) a.Y[yb + (long long)nl * HoWo] = acc[i][j][r2] + (a.bias && n < a.N ? a.bias[n] : 0.f);
      }
  }
}
