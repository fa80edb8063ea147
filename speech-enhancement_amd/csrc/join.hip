// Decoder skip join (models/_2206_07293_frcrn.py:93-100): align the decoder
// state x to the skip's grid (drop trailing time columns, frcrn.py:95-96;
// zero-pad trailing frequency rows, :97-98) and complex-concatenate
// (complex_nn.py:4-16: [x_re, s_re, x_im, s_im]).
//
// The PyTorch formulation costs ~11 activation-sized passes per decoder layer
// (slice, pad copy, chunk + cat forward; chunk-backward cats, slice_backward
// zero-fill + copy and .contiguous() copies backward). Here the forward is one
// read of (x, s) and one write of the joined tensor, and the backward one read
// of its gradient and one write of (dx, ds) — dx carries the zeros of the
// dropped columns, so no separate fill.
//
// Layout: contiguous NCHW, complex channel-stacked. x [B, Cx, Fx, Tx],
// s [B, Cs, F, T], out [B, Cx + Cs, F, T]; x is cropped / zero-padded at the
// END of each spatial dim.
#include "common.hpp"

namespace {

constexpr int kThreads = 256;

struct JoinGeom {
  int B, Cx, Fx, Tx, Cs, F, T;
};

// joined channel o -> (source 0 = x / 1 = s, source channel)
__device__ __forceinline__ void join_src(const JoinGeom& g, int o, int& src, int& c) {
  const int hx = g.Cx / 2, hs = g.Cs / 2;
  if (o < hx) { src = 0; c = o; }
  else if (o < hx + hs) { src = 1; c = o - hx; }
  else if (o < 2 * hx + hs) { src = 0; c = hx + (o - hx - hs); }
  else { src = 1; c = hs + (o - 2 * hx - hs); }
}

// One block per joined plane (b, o): rows f, lanes along t (coalesced).
// grid (B * (Cx + Cs))
__global__ __launch_bounds__(kThreads) void join_fwd_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                            float* __restrict__ out, JoinGeom g) {
  const int Co = g.Cx + g.Cs;
  const int b = blockIdx.x / Co, o = blockIdx.x - b * Co;
  int src, c;
  join_src(g, o, src, c);
  float* op = out + ((long long)b * Co + o) * g.F * g.T;
  if (src == 1) {
    const float* sp = s + ((long long)b * g.Cs + c) * g.F * g.T;
    for (int i = threadIdx.x; i < g.F * g.T; i += kThreads) op[i] = sp[i];   // same grid: flat copy
    return;
  }
  const float* xp = x + ((long long)b * g.Cx + c) * g.Fx * g.Tx;
  for (int f = 0; f < g.F; ++f)
    for (int t = threadIdx.x; t < g.T; t += kThreads)
      op[f * g.T + t] = (f < g.Fx && t < g.Tx) ? xp[f * g.Tx + t] : 0.f;
}

// dx over x's own grid (zeros where x was cropped away), ds = its slots.
// grid (B * (Cx + Cs))
__global__ __launch_bounds__(kThreads) void join_bwd_kernel(const float* __restrict__ gout, float* __restrict__ gx,
                                                            float* __restrict__ gs, JoinGeom g) {
  const int Co = g.Cx + g.Cs;
  const int b = blockIdx.x / Co, o = blockIdx.x - b * Co;
  int src, c;
  join_src(g, o, src, c);
  const float* gp = gout + ((long long)b * Co + o) * g.F * g.T;
  if (src == 1) {
    float* sp = gs + ((long long)b * g.Cs + c) * g.F * g.T;
    for (int i = threadIdx.x; i < g.F * g.T; i += kThreads) sp[i] = gp[i];
    return;
  }
  float* xp = gx + ((long long)b * g.Cx + c) * g.Fx * g.Tx;
  for (int f = 0; f < g.Fx; ++f)
    for (int t = threadIdx.x; t < g.Tx; t += kThreads)
      xp[f * g.Tx + t] = (f < g.F && t < g.T) ? gp[f * g.T + t] : 0.f;
}

int check(const JoinGeom& g) {
  if (g.B <= 0 || g.Cx <= 0 || g.Cs <= 0 || g.Fx <= 0 || g.Tx <= 0 || g.F <= 0 || g.T <= 0) return SE_E_ARG;
  if ((g.Cx & 1) || (g.Cs & 1)) return SE_E_SHAPE;
  if ((long long)g.B * (g.Cx + g.Cs) > 0x7fffffffll) return SE_E_SHAPE;
  if ((long long)g.F * g.T >= (1ll << 31) || (long long)g.Fx * g.Tx >= (1ll << 31)) return SE_E_SHAPE;
  return SE_OK;
}

}  // namespace

extern "C" int se_complex_join(const float* x, int Cx, int Fx, int Tx, const float* s, int Cs, int F, int T,
                               float* out, int B, void* stream) {
  JoinGeom g{B, Cx, Fx, Tx, Cs, F, T};
  if (int rc = check(g)) return rc;
  if (!x || !s || !out) return SE_E_ARG;
  dim3 grid(B * (Cx + Cs));
  hipLaunchKernelGGL(join_fwd_kernel, grid, dim3(kThreads), 0, se::as_stream(stream), x, s, out, g);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_complex_join_bwd(const float* gout, float* gx, int Cx, int Fx, int Tx, float* gs, int Cs, int F,
                                   int T, int B, void* stream) {
  JoinGeom g{B, Cx, Fx, Tx, Cs, F, T};
  if (int rc = check(g)) return rc;
  if (!gout || !gx || !gs) return SE_E_ARG;
  dim3 grid(B * (Cx + Cs));
  hipLaunchKernelGGL(join_bwd_kernel, grid, dim3(kThreads), 0, se::as_stream(stream), gout, gx, gs, g);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
