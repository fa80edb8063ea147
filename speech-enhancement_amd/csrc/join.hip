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

// Plane copy of n elements: 16-B vectors when both planes start 16-B aligned (the
// element count of a plane decides it, the same for every plane of a launch), scalars
// for the tail and otherwise.
template <typename E>
__device__ __forceinline__ void copy_plane(E* __restrict__ d, const E* __restrict__ s, long long n) {
  constexpr int V = 16 / sizeof(E);
  long long done = 0;
  if (((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15) == 0) {
    const long long nv = n / V;
    for (long long i = threadIdx.x; i < nv; i += kThreads)
      reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
    done = nv * V;
  }
  for (long long i = done + threadIdx.x; i < n; i += kThreads) d[i] = s[i];
}

// rows [0, rows_out) of width w_out from rows of width w_in (rows >= rows_in and
// columns >= w_in read 0): one wave per row, lanes along the row
template <typename E>
__device__ __forceinline__ void copy_rows(E* __restrict__ d, int rows_out, int w_out, const E* __restrict__ s,
                                          int rows_in, int w_in) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int f = wave; f < rows_out; f += kThreads / 64) {
    E* dr = d + (long long)f * w_out;
    if (f < rows_in) {
      const E* sr = s + (long long)f * w_in;
      for (int t = lane; t < w_out; t += 64) dr[t] = t < w_in ? sr[t] : E(0);
    } else {
      for (int t = lane; t < w_out; t += 64) dr[t] = E(0);
    }
  }
}

// One block per joined plane (b, o). E: the element's bit pattern (fp32, or bf16 /
// fp16 storage: a copy moves bits, and a zero is all-zero bits in every format).
// grid (B * (Cx + Cs))
template <typename E>
__global__ __launch_bounds__(kThreads) void join_fwd_kernel(const E* __restrict__ x, const E* __restrict__ s,
                                                            E* __restrict__ out, JoinGeom g) {
  const int Co = g.Cx + g.Cs;
  const int b = blockIdx.x / Co, o = blockIdx.x - b * Co;
  int src, c;
  join_src(g, o, src, c);
  E* op = out + ((long long)b * Co + o) * g.F * g.T;
  if (src == 1)   // same grid: flat copy
    copy_plane(op, s + ((long long)b * g.Cs + c) * g.F * g.T, (long long)g.F * g.T);
  else
    copy_rows(op, g.F, g.T, x + ((long long)b * g.Cx + c) * g.Fx * g.Tx, g.Fx, g.Tx);
}

// dx over x's own grid (zeros where x was cropped away), ds = its slots.
// grid (B * (Cx + Cs))
template <typename E>
__global__ __launch_bounds__(kThreads) void join_bwd_kernel(const E* __restrict__ gout, E* __restrict__ gx,
                                                            E* __restrict__ gs, JoinGeom g) {
  const int Co = g.Cx + g.Cs;
  const int b = blockIdx.x / Co, o = blockIdx.x - b * Co;
  int src, c;
  join_src(g, o, src, c);
  const E* gp = gout + ((long long)b * Co + o) * g.F * g.T;
  if (src == 1)
    copy_plane(gs + ((long long)b * g.Cs + c) * g.F * g.T, gp, (long long)g.F * g.T);
  else
    copy_rows(gx + ((long long)b * g.Cx + c) * g.Fx * g.Tx, g.Fx, g.Tx, gp, g.F, g.T);
}

int check(const JoinGeom& g) {
  if (g.B <= 0 || g.Cx <= 0 || g.Cs <= 0 || g.Fx <= 0 || g.Tx <= 0 || g.F <= 0 || g.T <= 0) return SE_E_ARG;
  if ((g.Cx & 1) || (g.Cs & 1)) return SE_E_SHAPE;
  if ((long long)g.B * (g.Cx + g.Cs) > 0x7fffffffll) return SE_E_SHAPE;
  if ((long long)g.F * g.T >= (1ll << 31) || (long long)g.Fx * g.Tx >= (1ll << 31)) return SE_E_SHAPE;
  return SE_OK;
}

}  // namespace

extern "C" int se_complex_join(const void* x, int Cx, int Fx, int Tx, const void* s, int Cs, int F, int T,
                               void* out, int B, int dtype, void* stream) {
  JoinGeom g{B, Cx, Fx, Tx, Cs, F, T};
  if (int rc = check(g)) return rc;
  if (!x || !s || !out || dtype < SE_DTYPE_F32 || dtype > SE_DTYPE_F16) return SE_E_ARG;
  dim3 grid(B * (Cx + Cs));
  if (dtype == SE_DTYPE_F32)
    hipLaunchKernelGGL(join_fwd_kernel<unsigned>, grid, dim3(kThreads), 0, se::as_stream(stream),
                       (const unsigned*)x, (const unsigned*)s, (unsigned*)out, g);
  else
    hipLaunchKernelGGL(join_fwd_kernel<unsigned short>, grid, dim3(kThreads), 0, se::as_stream(stream),
                       (const unsigned short*)x, (const unsigned short*)s, (unsigned short*)out, g);
  SE_LAUNCH_CHECK();
  return SE_OK;
}

extern "C" int se_complex_join_bwd(const void* gout, void* gx, int Cx, int Fx, int Tx, void* gs, int Cs, int F,
                                   int T, int B, int dtype, void* stream) {
  JoinGeom g{B, Cx, Fx, Tx, Cs, F, T};
  if (int rc = check(g)) return rc;
  if (!gout || !gx || !gs || dtype < SE_DTYPE_F32 || dtype > SE_DTYPE_F16) return SE_E_ARG;
  dim3 grid(B * (Cx + Cs));
  if (dtype == SE_DTYPE_F32)
    hipLaunchKernelGGL(join_bwd_kernel<unsigned>, grid, dim3(kThreads), 0, se::as_stream(stream),
                       (const unsigned*)gout, (unsigned*)gx, (unsigned*)gs, g);
  else
    hipLaunchKernelGGL(join_bwd_kernel<unsigned short>, grid, dim3(kThreads), 0, se::as_stream(stream),
                       (const unsigned short*)gout, (unsigned short*)gx, (unsigned short*)gs, g);
  SE_LAUNCH_CHECK();
  return SE_OK;
}
