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
