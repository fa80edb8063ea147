// CL16 operands of the SE_MATH_F16X3 weight-grad — included by cconv.hip after
// cconv_x3.hpp, inside its anonymous namespace.
//
// The split-fp16 GEMMs of cconv_x3.hpp gather fp32 activations one dword per
// lane per (row, k), scale and split them in registers and write the hi / lo
// planes to LDS: ~3 VALU per element, re-done for every tap / k-tile that
// reads the element. Here the operand is split ONCE, by the packing pass below
// (or by a producer), into "CL16": channels-last fp16 planes
//   P[plane][b][h][w][c], plane 0 = hi = fp16(x s), plane 1 = lo = fp16(x s - hi),
// s the per-tensor power-of-two scale of SE_MATH_F16X3 (max|x| s < 2^14), so a
// (position, 8-channel) chunk of an operand is 16 contiguous bytes per plane.

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

typedef __attribute__((address_space(3))) void lds_void;

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
