// Packed-operand gather GEMM (SE_MATH_F16X3 forward and data-grad) — included
// by cconv.hip after cconv_x3.hpp, inside its anonymous namespace.
//
// The split-fp16 GEMM of cconv_x3.hpp gathers fp32 activations one dword per
// lane per (row, k), scales and splits them in registers and writes the hi / lo
// planes to LDS: ~3 VALU per element, re-done for every tap (10x per element),
// plus 16 dword loads and 4 ds_write_b128 per thread per K-step.
// Here the operand is split ONCE, by the packing pass below (or by a producer),
// into "CL16": channels-last fp16 planes
//   P[plane][b][h][w][c], plane 0 = hi = fp16(x s), plane 1 = lo = fp16(x s - hi),
// s the per-tensor power-of-two scale of SE_MATH_F16X3 (max|x| s < 2^14). One
// (position, tap, 32-channel) row of the A tile is then 64 contiguous bytes per
// plane, and the LDS image of cconv_x3.hpp ([plane][128 rows][4 x 16 B chunks],
// chunk c of row r at c ^ ((r >> 2) & 3)) is filled by LDS-DMA: 16-byte
// buffer_load ... lds per lane, the swizzle applied to the per-lane SOURCE
// address (the LDS destination of a wave-instruction is lane-linear), rows
// outside the input (padding, m >= M) read as zeros through an out-of-range
// voffset. The pre-tiled weight image (prep_class_x3_kernel<true>) is copied the
// same way. No register staging, no conversion and no ds_write in the K loop;
// the MFMA fragments, the 2-stage LDS ring and the epilogue are those of
// gather_x3_kernel.

// ---------------------------------------------------------------------------
// Packing: x [B, C, H, W] fp32 -> CL16 planes with the scale from *amax.
// grid (ceil(HW / 64), ceil(C / 64), B), 256 threads: a 64-channel x
// 64-position tile is read along positions (coalesced), transposed in LDS and
// written as 64 positions x 128 B per plane.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
pack_cl16_kernel(const float* __restrict__ x, int C, int HW, const float* amax, _Float16* __restrict__ out,
                 long long plane_elems) {
  __shared__ float t[64][65];
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const float s = pow2f(kF16Top - amax_exp(amax));
  const float* xb = x + (long long)b * C * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + ty * 16 + i, p = p0 + tx;
    t[ty * 16 + i][tx] = (c < C && p < HW) ? xb[(long long)c * HW + p] * s : 0.f;
  }
  __syncthreads();
  // each thread: 8 consecutive channels of one position, both planes (16 B each)
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int idx = threadIdx.x + 256 * r;        // 0..511 = 64 positions x 8 chunks
    const int p = idx >> 3, ch = (idx & 7) * 8;
    if (p0 + p >= HW || c0 + ch >= C) continue;
    typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
    f16x8v hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = t[ch + e][p];
      const _Float16 h = (_Float16)v;
      hi[e] = h;
      lo[e] = (_Float16)(v - (float)h);
    }
    const long long o = ((long long)b * HW + p0 + p) * C + c0 + ch;
    *reinterpret_cast<f16x8v*>(out + o) = hi;
    *reinterpret_cast<f16x8v*>(out + plane_elems + o) = lo;
  }
}

// ---------------------------------------------------------------------------
// Gather GEMM over CL16 operands: one 8-wave workgroup per CU, a BM x BN tile
// ((256, 128) for the 128-column passes, (128, 256) for the 256-column
// data-grad) of 64 x 64 wave tiles (the fragments of gather_x3_kernel), and a
// 3-stage LDS ring: the stage two K-steps ahead is issued by LDS-DMA before the
// current one is computed, then a COUNTED s_waitcnt vmcnt (this wave's loads of
// the next stage retired, the newest stage still in flight) and a raw s_barrier
// (not __syncthreads, whose vmcnt(0) would drain the in-flight stage) hand the
// next stage to every wave. MI355X_MICROARCH/cdna_hip_programming: the
// 2-barrier 128 x 128 structure of gather_x3_kernel sits at its ~900 TF issue
// ceiling; keeping the LDS-DMA in flight across the barrier is what moves past it.
// Requires the tap-uniform K order (Cg % 32 == 0). JM as gather_x3_kernel.
// a.X (and a.X2 for JM = 1) point at CL16 buffers; a.Cpk = channels per
// position of a.X, a.Cpk2 of a.X2; a.pk_plane / a.pk_plane2 = elements per plane.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kPkThreads = 512, kPkStages = 3;

// (BM, BN) = (256, 256), S = 2: 8 waves of 128 (m) x 64 (n), two 64-KB stages,
// the next stage issued before the current one is computed.
template <int JM, int BM, int BN, int S = kPkStages>
__global__ void __launch_bounds__(kPkThreads, 1)
gather_pk_kernel(const GatherArgs a) {
  static_assert((BM == 256 && BN == 128) || (BM == 128 && BN == 256) || (BM == 256 && BN == 256 && S == 2),
                "8 waves of 64 x 64, or of 128 x 64 with two stages");
  constexpr bool BIG = BM == 256 && BN == 256;
  constexpr int WM = BIG ? 2 : BM / 64, TN = 64, TM = BM / WM, RN = 2, RM = TM / 32, PL = 2;
  constexpr int A_U4 = BM * 2 * 4, B_U4 = BN * 2 * 4;      // u32x4 per stage image
  constexpr int A_PCS = BM / 64, B_PCS = BN / 64;           // 1-KB LDS-DMA pieces per wave per stage
  constexpr int VM_NEXT = A_PCS + B_PCS;                    // loads of one stage per wave
  // ONE LDS array: the stage ring (LDS-DMA targets), then the epilogue's bias. Nothing
  // else is read from memory inside the K loop: a K-step's tap and first channel come
  // from scalar arithmetic and the per-tap offsets from the kernel arguments (a table
  // read from global memory or LDS there is waited for with vmcnt(0), which would drain
  // the stage in flight)
  constexpr int RING = S * (A_U4 + B_U4);
  __shared__ __attribute__((aligned(16))) u32x4 smem_all[RING];
  auto stage_base = [&](int buf) __attribute__((always_inline)) { return &smem_all[buf * (A_U4 + B_U4)]; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int NT = gridDim.y;
  const int tile = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = a.Kp / kBK;

  const int ea = amax_exp(a.amax_a);
  const int ush = ea + amax_exp(a.amax_w) - 2 * kF16Top;

  auto uniform_ptr = [](const void* p) __attribute__((always_inline)) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (void*)(((unsigned long long)hi << 32) | lo);
  };
  // A pieces: g = A_PCS * wave + j covers plane g / (BM / 16), rows 16 (g % (BM / 16)) + lane / 4,
  // LDS slot lane & 3 (its source chunk carries the XOR swizzle)
  constexpr int PPP = BM / 16;                    // pieces per plane
  const int qhw = a.Qh * a.Qw;
  const int b0 = m0 / qhw;
  const int slot = lane & 3;
  int rbase[A_PCS], hb[A_PCS], wb[A_PCS], csrc[A_PCS], pln[A_PCS];
  bool rval[A_PCS];
#pragma unroll
  for (int j = 0; j < A_PCS; ++j) {
    const int g = A_PCS * wave + j;
    pln[j] = g / PPP;
    const int r = 16 * (g % PPP) + (lane >> 2);
    const int m = m0 + r;
    rval[j] = m < a.M;
    const int mm = rval[j] ? m : m0;
    const int b = mm / qhw, rr = mm - b * qhw;
    const int qh = rr / a.Qw, qw = rr - qh * a.Qw;
    hb[j] = qh * a.sh;
    wb[j] = qw * a.sw;
    rbase[j] = b - b0;
    csrc[j] = slot ^ x3_swz(r);
  }
  const long long HW1 = (long long)a.Hi * a.Wi, HW2 = (long long)a.H2 * a.W2;
  const _Float16* X = reinterpret_cast<const _Float16*>(a.X);
  const _Float16* X2 = reinterpret_cast<const _Float16*>(a.X2);
  // per plane (a wave's A pieces may straddle the two planes when A_PCS = 2 and BM = 128)
  __amdgpu_buffer_rsrc_t rx[2], rx2[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    rx[p] = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(X + (p ? a.pk_plane : 0) + (long long)b0 * HW1 * a.Cpk),
                                              (short)0, 0x7FFFFFFF, 0x00020000);
    rx2[p] = rx[p];
    if constexpr (JM == 1)
      rx2[p] = __builtin_amdgcn_make_buffer_rsrc(
          uniform_ptr(X2 + (p ? a.pk_plane2 : 0) + (long long)b0 * HW2 * a.Cpk2), (short)0, 0x7FFFFFFF, 0x00020000);
  }
  // this workgroup's BN / 128 consecutive weight images of a K-step
  const u32x4* wt = reinterpret_cast<const u32x4*>(a.Wp) + (long long)nt * (BN / 128) * kX3TileU4;
  const int NTW = NT * (BN / 128);                // 128-column images per K-step

  auto stage = [&](int buf, int k0) __attribute__((always_inline)) {
    int t, c0;                                    // the step's tap and first channel (uniform)
    split_k(k0, a.Cg, a.ntaps, a.kblk, t, c0);
    const int offh = a.toffh[t], offw = a.toffw[t];
    int W = a.Wi, C = a.Cpk;
    long long HWs = HW1;
    bool from_x = false;
    if constexpr (JM == 1) {                      // a K-step lies in one join chunk
      const int q = c0 / a.jh;
      from_x = (q & 1) == 0;                      // chunks [x_re, s_re, x_im, s_im]
      c0 = (q >> 1) * a.jh + (c0 - q * a.jh);
      if (from_x) { W = a.W2; C = a.Cpk2; HWs = HW2; }
    }
    char* dstA = (char*)stage_base(buf);
#pragma unroll
    for (int j = 0; j < A_PCS; ++j) {
      const int hi = hb[j] + offh, wi = wb[j] + offw;
      bool ok = rval[j] & ((unsigned)hi < (unsigned)a.Hi) & ((unsigned)wi < (unsigned)a.Wi);
      if constexpr (JM == 1) ok &= !from_x | (hi < a.H2);   // F.pad rows of x read 0
      const int pos = (int)((long long)rbase[j] * HWs + (long long)hi * W + wi);
      const int vo = ok ? (pos * C + c0 + 8 * csrc[j]) * 2 : (int)0x80000000;
      __amdgpu_buffer_rsrc_t r = pln[j] ? (from_x ? rx2[1] : rx[1]) : (from_x ? rx2[0] : rx[0]);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(dstA + (A_PCS * wave + j) * 1024), 16, vo, 0, 0, 0);
    }
    const u32x4* src = wt + (long long)(k0 >> 5) * NTW * kX3TileU4 + (B_PCS * wave) * 64 + lane;
    char* dstB = (char*)(stage_base(buf) + A_U4);
#pragma unroll
    for (int j = 0; j < B_PCS; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(src + 64 * j),
                                       (lds_void*)(dstB + (B_PCS * wave + j) * 1024), 16, 0, 0);
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
  constexpr int FS = BIG ? 1 : 2;                  // k-substeps of fragments held at once
  auto compute = [&](int cur) __attribute__((always_inline)) {
    const u32x4* sA = stage_base(cur);
    const u32x4* sW = stage_base(cur) + A_U4;
#pragma unroll
    for (int k0 = 0; k0 < 2; k0 += FS) {
      u32x4 wf[FS][RN][PL], af[FS][RM][PL];
#pragma unroll
      for (int kk = 0; kk < FS; ++kk) {
        const int c = (2 * (k0 + kk) + lh) ^ fsw;
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          const int n = wn * TN + 32 * i;         // block's first column (uniform)
#pragma unroll
          for (int p = 0; p < PL; ++p)
            wf[kk][i][p] = sW[(((n >> 7) * PL + p) * 128 + (n & 127) + lr) * 4 + c];
        }
#pragma unroll
        for (int j = 0; j < RM; ++j)
#pragma unroll
          for (int p = 0; p < PL; ++p)
            af[kk][j][p] = sA[(p * BM + wm * TM + 32 * j + lr) * 4 + c];
      }
      if constexpr (BIG) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < FS; ++kk)
#pragma unroll
        for (int t = 0; t < 3; ++t)  // hi*hi, hi*lo, lo*hi
#pragma unroll
          for (int i = 0; i < RN; ++i)
#pragma unroll
            for (int j = 0; j < RM; ++j)
              acc[i][j] = mfma_32x32x16<true>(wf[kk][i][t == 2 ? 1 : 0], af[kk][j][t == 1 ? 1 : 0], acc[i][j]);
      if constexpr (BIG) __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (S == 2) {
    // prologue: stage 0; each K-step issues the next stage, computes, then waits for it
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * kBK);
      compute(kt & 1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    // prologue: stages 0 and 1 in flight, wait for stage 0
    stage(0, 0);
    if (nk > 1) stage(1, kBK);
    if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(VM_NEXT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const bool ahead = kt + 2 < nk;
      if (ahead) stage((kt + 2) % S, (kt + 2) * kBK);
      compute(kt % S);
      // retire this wave's loads of stage kt + 1 (the stage kt + 2 ones may stay in flight),
      // then the barrier hands stage kt + 1 to every wave and frees buffer kt for kt + 3
      if (ahead) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(VM_NEXT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], ush);

  // --- epilogue (as gather_x3_kernel) ---
  float* sBias = reinterpret_cast<float*>(&smem_all[0]);
  for (int i = tid; i < BN; i += kPkThreads) {
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
    const int b = mm / qhw, r = mm - b * qhw;
    const int qh = r / a.Qw, qw = r - qh * a.Qw;
    const int nl0 = wn * TN + 4 * lh;
    if constexpr (JM == 2) {
      const int oh = a.ph + a.Sh * qh, ow = a.pw + a.Sw * qw;
      const long long P2 = (long long)a.YH2 * a.YW2;
      const int cpb = 2 * a.yjh;
#pragma unroll
      for (int i = 0; i < RN; ++i) {
        const int nb = n0 + wn * TN + 32 * i;     // block's first channel (wave-uniform)
        const int q = nb / a.yjh;
        const int cb = (q >> 1) * a.yjh + (nb - q * a.yjh) + 4 * lh;
        const bool to_x = (q & 1) == 0;
        if (to_x && oh >= a.YH2) continue;
        const long long pl = to_x ? P2 : HoWo;
        float* yp = to_x ? a.Y2 + ((long long)b * cpb + cb) * P2 + (long long)oh * a.YW2 + ow
                         : a.Y + ((long long)b * cpb + cb) * HoWo + (long long)oh * a.Wo + ow;
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) yp[(long long)((r2 & 3) + 8 * (r2 >> 2)) * pl] = acc[i][j][r2];
      }
      continue;
    }
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

// ---------------------------------------------------------------------------
// Weight-grad over CL16 operands: dWp[k, n] = sum_m G[m, k] D[m, n] with the
// tap-major K order of the weight-grad (a 128-row k-tile is 128 channels of one
// tap), so in CL16 form a (position, tap) row of G and a position row of D are
// each one contiguous 256-B segment per plane: exactly a row of the [position]
// [128 rows] LDS image of wgrad_x3_kernel (XOR chunk swizzle wx3_off). Each
// m-step is 32 consecutive positions of ONE output row (b, qh): the row's
// positions qw0 .. qw0 + 31 (the last step of a row is partial, ~3 % padding at
// Qw = 403), so the tap offset and bounds are uniform per step. Wave w stages
// one plane of one operand for all 32 positions with 8 x 16-B global_load_lds
// per lane (per-lane addresses: the joined D's chunks come from x or s per
// lane; invalid lanes read the zeroed workspace page). 2-stage ring, the
// fragments (ds_read_b64_tr_b16), MFMA terms and slab output of wgrad_x3_kernel.
// a.X = CL16 G (Cg channels on Hi x Wi), a.D = CL16 D (N channels on Qh x Qw)
// or, DJ, CL16 s with D2 = CL16 x (djh-channel chunks [x_re, s_re, x_im, s_im]).
// a.m_per_split = output rows (b, qh) per split.
// ---------------------------------------------------------------------------
template <bool DJ>
__global__ void __launch_bounds__(kThreads, 2)
wgrad_pk_kernel(const WgradArgs a) {
  constexpr int BKO = 128, BNO = 128, WNn = 2, TK = 64, TN = 64, RK = 2, RN = 2, BMR = 32;
  constexpr int PLANE = BMR * 256;           // bytes of one [32 positions][128 rows] f16 plane
  __shared__ __attribute__((aligned(16))) unsigned char sm[2][4 * PLANE];   // G hi, G lo, D hi, D lo

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave / WNn, wnn = wave % WNn;
  const int nkn = gridDim.x * gridDim.y;
  const int tile = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, nkn * gridDim.z);
  const int split = tile / nkn, kn = tile % nkn;
  const int k0 = (kn % gridDim.x) * BKO, n0 = (kn / gridDim.x) * BNO;
  const int rows = (a.M / a.Qw);             // = B * Qh output rows
  const int rbeg = split * a.m_per_split;
  const int rend = min(rows, rbeg + a.m_per_split);
  const int spr = (a.Qw + BMR - 1) / BMR;    // m-steps per row
  const int nsteps = rend > rbeg ? (rend - rbeg) * spr : 0;

  const int eg = amax_exp(a.amax_g), ed = amax_exp(a.amax_d);
  const int ush = eg + ed - 2 * kF16Top;
  // tap of this k-tile (tap-major K order, Cg % 128 == 0) and its first channel
  const int tap = k0 / a.Cg, cbase = k0 - tap * a.Cg;
  const int offh = a.toffh[tap], offw = a.toffw[tap];

  const _Float16* G = reinterpret_cast<const _Float16*>(a.X);
  const _Float16* Dp = reinterpret_cast<const _Float16*>(a.D);
  const _Float16* D2p = reinterpret_cast<const _Float16*>(a.D2);
  const _Float16* zero = reinterpret_cast<const _Float16*>(a.zero);
  // this wave's operand / plane; this lane's position (s = 4 j + lane / 16) and LDS slot
  const bool isG = wave < 2;
  const int plane = wave & 1;
  const int sl = lane & 15, s0 = lane >> 4;
  const long long HiWi = (long long)a.Hi * a.Wi, QQ = (long long)a.Qh * a.Qw, QQ2 = (long long)a.DH2 * a.DW2;

  auto stage = [&](int buf, int step) __attribute__((always_inline)) {
    const int row = rbeg + step / spr;
    const int qw0 = (step - (step / spr) * spr) * BMR;
    const int b = row / a.Qh, qh = row - b * a.Qh;
    const int hg = qh * a.sh + offh;            // G input row of the tap (uniform)
    unsigned char* dst = sm[buf] + (isG ? plane : 2 + plane) * PLANE;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int s = 4 * j + s0;                   // position row of the LDS image
      const int ch = sl ^ wx3_swz(s);   // source chunk (16 B = 8 channels)
      const int qw = qw0 + s;
      const _Float16* src = zero;
      if (isG) {
        const int wg = qw * a.sw + offw;
        const bool ok = (qw < a.Qw) & ((unsigned)hg < (unsigned)a.Hi) & ((unsigned)wg < (unsigned)a.Wi);
        if (ok) src = G + (plane ? a.pk_plane_g : 0) + (((long long)b * HiWi + (long long)hg * a.Wi + wg) * a.Cg
                                                          + cbase + 8 * ch);
      } else if constexpr (DJ) {
        const int jc = n0 + 8 * ch;               // joined channel
        const int q = jc / a.djh;
        const bool from_x = (q & 1) == 0;         // chunks [x_re, s_re, x_im, s_im]
        const int c = (q >> 1) * a.djh + (jc - q * a.djh);
        const int cpb = 2 * a.djh;
        const bool ok = (qw < a.Qw) & (!from_x | (qh < a.DH2));   // F.pad rows of x: 0
        if (ok)
          src = from_x ? D2p + (plane ? a.pk_plane_d2 : 0) + (((long long)b * QQ2 + (long long)qh * a.DW2 + qw) * cpb + c)
                       : Dp + (plane ? a.pk_plane_d : 0) + (((long long)b * QQ + (long long)qh * a.Qw + qw) * cpb + c);
      } else {
        const bool ok = qw < a.Qw;
        if (ok) src = Dp + (plane ? a.pk_plane_d : 0) + (((long long)b * QQ + (long long)qh * a.Qw + qw) * a.N
                                                           + n0 + 8 * ch);
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + j * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[RK][RN];
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int g = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
  auto frag = [&](const unsigned char* pl, int row0, int pos0) __attribute__((always_inline)) {
    const int c0 = (row0 + 16 * (g & 1)) >> 3;
    const int s = pos0 + 8 * (g >> 1) + gq;
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(pl + wx3_off(s, c0 + (gp >> 1)) + 8 * (gp & 1)));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(pl + wx3_off(s + 4, c0 + (gp >> 1)) + 8 * (gp & 1)));
    return __builtin_bit_cast(u32x4, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int cur) __attribute__((always_inline)) {
    const unsigned char* base = sm[cur];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 ga[RK][2], gb[RN][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int i = 0; i < RK; ++i) ga[i][p] = frag(base + p * PLANE, wk * TK + 32 * i, 16 * ks);
#pragma unroll
        for (int j = 0; j < RN; ++j) gb[j][p] = frag(base + (2 + p) * PLANE, wnn * TN + 32 * j, 16 * ks);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < RK; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = mfma_32x32x16<true>(ga[i][t == 2 ? 1 : 0], gb[j][t == 1 ? 1 : 0], acc[i][j]);
    }
  };

  if (nsteps > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) stage((s + 1) & 1, s + 1);
      compute(s & 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
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
        out[(long long)k * a.Np + n] = __builtin_ldexpf(acc[i][j][r], ush);
      }
}
