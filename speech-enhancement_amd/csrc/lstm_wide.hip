// Wide-hidden LSTM recurrence (H = 256 / 512 / 1024): CARN's nn.LSTM(512, 512,
// 2 layers) (models/_2104_05267_carn.py:132; config 5 runs it over 9002
// frames), CRN's nn.LSTM(1024, 1024, 2 layers) (models/_1809_01405_crn.py:90)
// and any ComplexLSTM / nn.LSTM of those widths. Same contract and layouts as
// lstm.hip (torch.nn.LSTM math, gate order i, f, g, o, h0 = c0 = 0; xproj and
// all weight gradients are the caller's GEMMs), different decomposition:
//
// W_hh is 4H x H fp32 = 1 / 4 / 16 MB: more than one CU's register file. A
// GROUP of NWG = H / U workgroups runs one block of BS sequences of one LSTM;
// member m owns hidden units [U m, U m + U) (U = 32, or 16 at H = 1024 so that
// a thread still holds 128 weights):
//   fwd: the 4U gate rows of its units (4U x H weights in VGPRs, thread = one
//        row x one 1/QS of the columns, QS = 512 / 4U), the cell update of its
//        units;
//   bwd: the U columns of its units over all 4H rows (4H x U weights, thread =
//        one column x one 1/RBN of the rows, RBN = 512 / U), the cell backward
//        of its units.
// Per step the members exchange h_t (fwd, H floats per sequence) or dgates_t
// (bwd, 4H floats per sequence) through the h / dgates OUTPUTS themselves:
// agent-scope atomic stores and loads (coherent across XCDs and CUs), and one
// monotonically increasing counter per group (target NWG * (step + 1)). Every
// address is written once and read after the counter says so.
//
// Residency: a group's members spin on each other, so all of them must be
// resident together; the host admits a launch only when every group fits on
// the device at one workgroup per CU, and runs larger batches as consecutive
// launches over batch slices. Sync groups of up to 32 members are placed on
// one XCD each (block id % 8 is the XCD under round-robin dispatch, so the
// exchange stays in one L2 where the placement holds); a 64-member group
// (H = 1024) spans two XCDs. The spin is bounded: on a timeout the workgroup
// stops waiting, writes NaN outputs from then on and sets *status.
#include "common.hpp"

namespace {

constexpr int kWThreads = 512;
constexpr int kMaxSpins = 1 << 24;         // x s_sleep(1) (64 clk): ~0.4 s

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float ld_agent(const float* p) {
  return __int_as_float(__hip_atomic_load(reinterpret_cast<const int*>(p), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<int*>(p), __float_as_int(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float tanh_w(float x) {   // branch-free (see lstm.hip tanh_bf)
  const float ax = fabsf(x), x2 = x * x;
  const float e = expf(-2.f * ax);
  const float big = copysignf((1.f - e) / (1.f + e), x);
  const float small = x * (1.f + x2 * (-1.f / 3.f + x2 * (2.f / 15.f + x2 * (-17.f / 315.f))));
  return ax < 0.0625f ? small : big;
}

struct WideArgs {
  const float* xproj;   // fwd
  const float* w_hh;    // [L][4H][H]
  const float* dy;      // bwd
  float* h;
  float* c;
  float* gates;
  float* dgates;
  long long x_lstm;
  int x_row;
  int B, T;
  unsigned rev_mask;
  int ngroups, nbg;     // groups; batch groups per LSTM
  int b_lo, b_hi;       // the batch slice [b_lo, b_hi) this launch runs
  int* sync;            // [ngroups] step counters (zeroed by the host)
  int* status;
};

// block -> (group, member): a group's members share block id % 8 (one XCD),
// or for NWG > 32 spread over XPG = NWG / 32 consecutive XCD ids
template <int NWG>
__device__ __forceinline__ void role_of(int bid, int& gi, int& mem) {
  constexpr int XPG = NWG > 32 ? NWG / 32 : 1, MPX = NWG / XPG;
  const int xcd = bid & 7, slot = bid >> 3;
  gi = xcd / XPG + (8 / XPG) * (slot / MPX);
  mem = (xcd % XPG) * MPX + slot % MPX;
}

// Publish this workgroup's stores of the step, arrive, wait for the group.
// Every storing thread has waited for its own stores (vmcnt(0)) before the
// barrier; thread 0 then arrives and spins. Returns false once timed out.
__device__ __forceinline__ bool group_barrier(int* ctr, int target, bool ok, int* status, int* s_ok) {
  __builtin_amdgcn_s_waitcnt(0x0F70 | 0);   // vmcnt(0): this thread's stores are performed
  __syncthreads();
  if (threadIdx.x == 0) {
    bool good = ok;
    if (good) {
      __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kMaxSpins) {
          good = false;
          __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    *s_ok = good ? 1 : 0;
  }
  __syncthreads();
  return *s_ok != 0;
}

template <int H, int U, int BS>
__global__ __launch_bounds__(kWThreads) void lstmw_fwd_kernel(WideArgs a) {
  constexpr int NWG = H / U, G = 4 * H, R = 4 * U, QS = kWThreads / R, KQ = H / QS, RW = R / 64;
  static_assert(R % 64 == 0 && KQ % 4 == 0 && KQ <= 128, "fwd thread map");
  int gi, mem;
  role_of<NWG>(blockIdx.x, gi, mem);
  if (gi >= a.ngroups) return;                      // whole padding groups leave together
  const int l = gi / a.nbg, b0 = a.b_lo + (gi % a.nbg) * BS;
  const int j0 = mem * U;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = (wave % RW) * 64 + lane;          // local gate row: gate row / U, unit row % U
  const int q = __builtin_amdgcn_readfirstlane(wave / RW);   // column part
  const bool rev = (a.rev_mask >> l) & 1u;
  const int T = a.T, dir = rev ? -1 : 1, t0 = rev ? T - 1 : 0;

  f32x2 w[KQ / 2];
  {
    const int grow = (row / U) * H + j0 + (row % U);
    const float4* W = reinterpret_cast<const float4*>(a.w_hh + ((size_t)l * G + grow) * H + q * KQ);
#pragma unroll
    for (int k = 0; k < KQ / 4; ++k) {
      const float4 v = W[k];
      w[2 * k] = f32x2{v.x, v.y};
      w[2 * k + 1] = f32x2{v.z, v.w};
    }
  }
  __shared__ __attribute__((aligned(16))) float sh[BS][H];   // h_{t-1}
  __shared__ float sp[QS][BS][R];                            // column-part partial sums
  __shared__ float sg[BS][R];                                // activated gates
  __shared__ int s_ok;
  for (int i = tid; i < BS * H; i += kWThreads) (&sh[0][0])[i] = 0.f;

  // gate threads: (b, r) = idx / R, idx % R for idx = tid + 512 u
  constexpr int GU = (BS * R + kWThreads - 1) / kWThreads;
  float xnext[GU];
  auto xrow = [&](int b, int r, int t) __attribute__((always_inline)) {
    const int bb = min(b0 + b, a.b_hi - 1);
    return a.xproj + (size_t)l * a.x_lstm + ((size_t)bb * T + t) * a.x_row + (r / U) * H + j0 + (r % U);
  };
  auto xfetch = [&](int s) __attribute__((always_inline)) {
    const int t = t0 + dir * min(s, T - 1);
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int idx = tid + kWThreads * u;
      xnext[u] = idx < BS * R ? *xrow(idx / R, idx % R, t) : 0.f;
    }
  };
  xfetch(0);
  float cst = 0.f;                                  // cell state of (b, j) = (tid / 32, tid % 32)
  const int cb = tid / U, cj = tid % U;
  bool ok = true;
  int* ctr = a.sync + gi;
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = t0 + dir * s;
    // recurrent products over this thread's quarter of h_{t-1}
    {
      f32x2 acc[BS][2];
#pragma unroll
      for (int b = 0; b < BS; ++b) acc[b][0] = acc[b][1] = f32x2{0.f, 0.f};
#pragma unroll
      for (int b = 0; b < BS; ++b) {
        const float4* hp = reinterpret_cast<const float4*>(&sh[b][q * KQ]);
#pragma unroll
        for (int k = 0; k < KQ / 4; ++k) {
          const float4 hv = hp[k];                 // LDS broadcast
          acc[b][0] = __builtin_elementwise_fma(w[2 * k], f32x2{hv.x, hv.y}, acc[b][0]);
          acc[b][1] = __builtin_elementwise_fma(w[2 * k + 1], f32x2{hv.z, hv.w}, acc[b][1]);
        }
      }
#pragma unroll
      for (int b = 0; b < BS; ++b) sp[q][b][row] = (acc[b][0].x + acc[b][0].y) + (acc[b][1].x + acc[b][1].y);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int idx = tid + kWThreads * u;
      if (idx < BS * R) {
        const int b = idx / R, r = idx % R;
        float rec = 0.f;
#pragma unroll
        for (int p = 0; p < QS; p += 2) rec += sp[p][b][r] + sp[p + 1][b][r];
        const float z = xnext[u] + rec;
        const float v = (r / U) == 2 ? tanh_w(z) : sigm(z);
        sg[b][r] = v;
        if (b0 + b < a.b_hi)
          a.gates[(((size_t)l * a.B + b0 + b) * T + t) * G + (r / U) * H + j0 + (r % U)] = ok ? v : __int_as_float(0x7fc00000);
      }
    }
    xfetch(s + 1);
    __syncthreads();
    if (tid < BS * U && b0 + cb < a.b_hi) {
      const float ig = sg[cb][cj], fg = sg[cb][U + cj], gg = sg[cb][2 * U + cj], og = sg[cb][3 * U + cj];
      cst = fg * cst + ig * gg;
      const size_t o = (((size_t)l * a.B + b0 + cb) * T + t) * H + j0 + cj;
      const float nan = __int_as_float(0x7fc00000);
      a.c[o] = ok ? cst : nan;
      st_agent(a.h + o, ok ? og * tanh_w(cst) : nan);
    }
    if (s + 1 == T) break;
    ok = group_barrier(ctr, NWG * (s + 1), ok, a.status, &s_ok);
    // h_t of every member -> sh (rows past B read as 0)
    for (int i = tid; i < BS * H; i += kWThreads) {
      const int b = i / H, k = i % H;
      (&sh[0][0])[i] = b0 + b < a.b_hi ? ld_agent(a.h + (((size_t)l * a.B + b0 + b) * T + t) * H + k) : 0.f;
    }
    __syncthreads();
  }
}

template <int H, int U, int BS>
__global__ __launch_bounds__(kWThreads) void lstmw_bwd_kernel(WideArgs a) {
  constexpr int NWG = H / U, G = 4 * H, RBN = kWThreads / U, RB = G / RBN;
  static_assert(RB % 4 == 0 && RB <= 128, "bwd thread map");
  int gi, mem;
  role_of<NWG>(blockIdx.x, gi, mem);
  if (gi >= a.ngroups) return;
  const int l = gi / a.nbg, b0 = a.b_lo + (gi % a.nbg) * BS;
  const int j0 = mem * U;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane % U;                         // unit j0 + col
  const int rb = wave * (64 / U) + lane / U;        // row block: rows rb*RB .. +RB of all 4H
  const bool rev = (a.rev_mask >> l) & 1u;
  const int T = a.T, dir = rev ? -1 : 1, t0 = rev ? T - 1 : 0;

  f32x2 w[RB / 2];
  {
    const float* W = a.w_hh + ((size_t)l * G + rb * RB) * H + j0 + col;
#pragma unroll
    for (int i = 0; i < RB / 2; ++i) w[i] = f32x2{W[(size_t)(2 * i) * H], W[(size_t)(2 * i + 1) * H]};
  }
  __shared__ __attribute__((aligned(16))) float sdg[BS][G];   // dgates_{t+1} of every member
  __shared__ float sp[RBN][BS][U];
  __shared__ int s_ok;
  for (int i = tid; i < BS * G; i += kWThreads) (&sdg[0][0])[i] = 0.f;

  // cell threads: (b, j) = (tid / U, tid % U), tid < BS * U
  const int cb = tid / U, cj = tid % U;
  const bool cell = tid < BS * U && b0 + cb < a.b_hi;
  const size_t rowc = ((size_t)l * a.B + min(b0 + cb, a.b_hi - 1)) * T;
  struct Pre { float dy, c, cp, g[4]; };
  auto fetch = [&](int s, Pre& p) __attribute__((always_inline)) {
    s = max(s, 0);
    const int t = t0 + dir * s, tp = t0 + dir * max(s - 1, 0);
    const size_t o = (rowc + t) * H + j0 + cj;
    p.dy = a.dy[o];
    p.c = a.c[o];
    p.cp = s > 0 ? a.c[(rowc + tp) * H + j0 + cj] : 0.f;
    const float* gp = a.gates + (rowc + t) * G + j0 + cj;
#pragma unroll
    for (int g = 0; g < 4; ++g) p.g[g] = gp[g * H];
  };
  Pre pre;
  if (cell) fetch(T - 1, pre);
  float dc = 0.f;
  bool ok = true;
  int* ctr = a.sync + gi;
  __syncthreads();

  for (int s = T - 1; s >= 0; --s) {
    const int t = t0 + dir * s;
    // dh_rec of this unit column: W_hh[:, j]^T dgates_{t+1} over this thread's row block
    {
      f32x2 acc[BS][2];
#pragma unroll
      for (int b = 0; b < BS; ++b) acc[b][0] = acc[b][1] = f32x2{0.f, 0.f};
#pragma unroll
      for (int b = 0; b < BS; ++b) {
        const float4* gp = reinterpret_cast<const float4*>(&sdg[b][rb * RB]);
#pragma unroll
        for (int i = 0; i < RB / 4; ++i) {
          const float4 gv = gp[i];
          acc[b][0] = __builtin_elementwise_fma(w[2 * i], f32x2{gv.x, gv.y}, acc[b][0]);
          acc[b][1] = __builtin_elementwise_fma(w[2 * i + 1], f32x2{gv.z, gv.w}, acc[b][1]);
        }
      }
#pragma unroll
      for (int b = 0; b < BS; ++b) sp[rb][b][col] = (acc[b][0].x + acc[b][0].y) + (acc[b][1].x + acc[b][1].y);
    }
    __syncthreads();
    if (cell) {
      float dh_rec = 0.f;
#pragma unroll
      for (int r = 0; r < RBN; ++r) dh_rec += sp[r][cb][cj];
      const Pre p = pre;
      if (s > 0) fetch(s - 1, pre);
      const float dh = p.dy + dh_rec, ct = p.c, cp = p.cp;
      const float ig = p.g[0], fg = p.g[1], gg = p.g[2], og = p.g[3];
      const float tc = tanh_w(ct);
      dc += dh * og * (1.f - tc * tc);
      const float nan = __int_as_float(0x7fc00000);
      float* dg = a.dgates + (rowc + t) * G + j0 + cj;
      st_agent(dg, ok ? dc * gg * ig * (1.f - ig) : nan);
      st_agent(dg + H, ok ? dc * cp * fg * (1.f - fg) : nan);
      st_agent(dg + 2 * H, ok ? dc * ig * (1.f - gg * gg) : nan);
      st_agent(dg + 3 * H, ok ? dh * tc * og * (1.f - og) : nan);
      dc *= fg;
    }
    if (s == 0) break;
    ok = group_barrier(ctr, NWG * (T - s), ok, a.status, &s_ok);
    for (int i = tid; i < BS * G; i += kWThreads) {
      const int b = i / G, r = i % G;
      (&sdg[0][0])[i] = b0 + b < a.b_hi ? ld_agent(a.dgates + (((size_t)l * a.B + b0 + b) * T + t) * G + r) : 0.f;
    }
    __syncthreads();
  }
}

struct Plan { int bs, nbg, ngroups, blocks; };

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return v;
  }();
  return n;
}

constexpr int units_of(int H) { return H > 512 ? 16 : 32; }

// Smallest BS whose groups take at most half the CUs (else all of them), for
// the batch slice of B sequences
int plan_of(int L, int B, int H, Plan& p) {
  const int nwg = H / units_of(H), cus = cu_count();
  const int gpr = nwg > 32 ? 8 / (nwg / 32) : 8;   // groups per round of 8 XCD ids
  if (cus <= 0) return SE_E_LAUNCH;
  for (int pass = 0; pass < 2; ++pass) {
    const int budget = pass == 0 ? cus / 2 : cus;
    for (int bs : {1, 2, 4, 8}) {
      const int nbg = (B + bs - 1) / bs;
      const long long wgs = (long long)L * nbg * nwg;
      if (wgs <= budget) {
        p.bs = bs; p.nbg = nbg; p.ngroups = L * nbg;
        p.blocks = ((p.ngroups + gpr - 1) / gpr) * gpr * nwg;
        return SE_OK;
      }
    }
  }
  return SE_E_UNSUPPORTED;
}

template <int H>
int launch_wide(bool bwd, WideArgs& a, const Plan& p, hipStream_t st) {
  constexpr int U = units_of(H);
  const dim3 grid(p.blocks), blk(kWThreads);
#define SE_WIDE_CASE(BSV)                                                                      \
  case BSV:                                                                                    \
    if (bwd) hipLaunchKernelGGL((lstmw_bwd_kernel<H, U, BSV>), grid, blk, 0, st, a);           \
    else hipLaunchKernelGGL((lstmw_fwd_kernel<H, U, BSV>), grid, blk, 0, st, a);               \
    break;
  switch (p.bs) {
    SE_WIDE_CASE(1)
    SE_WIDE_CASE(2)
    SE_WIDE_CASE(4)
    SE_WIDE_CASE(8)
    default: return SE_E_UNSUPPORTED;
  }
#undef SE_WIDE_CASE
  SE_LAUNCH_CHECK();
  return SE_OK;
}

// One launch per batch slice: the whole batch when its groups fit on the device
// at once, else slices of the largest multiple of 8 sequences that do.
int wide_common(bool bwd, WideArgs& a, int L, int H, int* sync, int* status, hipStream_t st) {
  if (L <= 0 || L > 32 || a.B <= 0 || a.T <= 0 || !sync || !status) return SE_E_ARG;
  if (H != 256 && H != 512 && H != 1024) return SE_E_UNSUPPORTED;
  if ((long long)L * a.B * a.T * 4 * H >= (1ll << 40)) return SE_E_SHAPE;
  Plan p{};
  int slice = a.B;
  while (plan_of(L, slice, H, p) != SE_OK) {
    if (slice <= 8) return SE_E_UNSUPPORTED;
    slice = ((slice / 2 + 7) / 8) * 8;
  }
  for (int lo = 0; lo < a.B; lo += slice) {
    const int nb = std::min(slice, a.B - lo);
    int rc = plan_of(L, nb, H, p);
    if (rc) return rc;
    a.ngroups = p.ngroups; a.nbg = p.nbg; a.sync = sync; a.status = status;
    a.b_lo = lo; a.b_hi = lo + nb;
    if (hipMemsetAsync(sync, 0, sizeof(int) * p.ngroups, st) != hipSuccess) return SE_E_LAUNCH;
    rc = H == 256 ? launch_wide<256>(bwd, a, p, st)
                  : H == 512 ? launch_wide<512>(bwd, a, p, st) : launch_wide<1024>(bwd, a, p, st);
    if (rc) return rc;
  }
  return SE_OK;
}

}  // namespace

extern "C" int se_lstm_wide_supported(int hidden) { return hidden == 256 || hidden == 512 || hidden == 1024; }

extern "C" int se_lstm_wide_sync_ints(void) { return 4096; }

extern "C" int se_lstm_wide_fwd(const float* xproj, long long x_lstm_stride, int x_row_stride, const float* w_hh,
                                float* h, float* c, float* gates, int L, int B, int T, int H, unsigned rev_mask,
                                int* sync, int* status, void* stream) {
  if (!xproj || !w_hh || !h || !c || !gates || x_row_stride < 4 * H) return SE_E_ARG;
  WideArgs a{};
  a.xproj = xproj; a.w_hh = w_hh; a.h = h; a.c = c; a.gates = gates;
  a.x_lstm = x_lstm_stride; a.x_row = x_row_stride; a.B = B; a.T = T; a.rev_mask = rev_mask;
  return wide_common(false, a, L, H, sync, status, se::as_stream(stream));
}

extern "C" int se_lstm_wide_bwd(const float* dy, const float* w_hh, const float* gates, const float* c,
                                float* dgates, int L, int B, int T, int H, unsigned rev_mask, int* sync,
                                int* status, void* stream) {
  if (!dy || !w_hh || !gates || !c || !dgates) return SE_E_ARG;
  WideArgs a{};
  a.dy = dy; a.w_hh = w_hh; a.gates = const_cast<float*>(gates); a.c = const_cast<float*>(c); a.dgates = dgates;
  a.B = B; a.T = T; a.rev_mask = rev_mask;
  return wide_common(true, a, L, H, sync, status, se::as_stream(stream));
}
