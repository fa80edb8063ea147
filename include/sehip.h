/*
 * sehip — MI355X-native complex-spectral enhancement ops (C ABI).
 *
 * This is the drop-in boundary for the hot path of shs2783/Speech-Enhancement
 * (SURVEY.md §8a/§8b). The reference has no FFI of its own: its "plugin API"
 * is the nn.Module surface of models/conv_stft.py and
 * models/modules/complex_nn.py. Each entry point below replaces the ATen
 * calls made at the cited reference line(s); the Python host package
 * (speech-enhancement_amd/sehip) mirrors the reference modules on top of it.
 *
 * Conventions
 *   - Plain pointers to device memory (fp32, contiguous NCHW / [B, F, T]).
 *   - Complex tensors are channel-stacked: channels [0, C/2) are the real
 *     parts, [C/2, C) the imaginary parts (complex_nn.py:18-42).
 *   - `stream` is a hipStream_t (the caller's current stream). Nothing here
 *     synchronises the device; all launches are asynchronous on `stream`.
 *   - The library allocates nothing. Scratch is passed in (`ws`, `ws_bytes`);
 *     query the size with the matching *_workspace_size function.
 *   - Return value: SE_OK (0) or a negative SE_E_* code; se_strerror() names it.
 */
#ifndef SEHIP_H
#define SEHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEHIP_ABI_VERSION 11  /* 11: se_cbn_bwd_ccbam (the CCBAM gate's input gradient formed inside the
                                 encoder CBN backward);
                                 10: 16-bit storage and row biases in se_gemm (the Linear layers), se_bias_grad,
                                 se_copy_strided, the CARN mask / attention-gate / clamp passes, the
                                 ComplexLSTM re/im combine, long-form chunking, 16-bit SI-SNR / clip / AdamW,
                                 the polar masks' leading zero rows;
                                 9: se_polar_mask_fwd / _bwd; 8: CL16 operands removed (se_pack_cl16*, se_conv2d_desc.x_packed /
                                 .x2_packed / .dy_packed / .x2_amax, se_cbn_fwd's y_packed,
                                 se_ccbam_apply's out_packed / out_amax: measured slower);
                                 7: measured-neutral variants removed (se_conv2d_desc.accumulate_dx /
                                 .moments, se_cbn_*_fwd_moments, se_stream_create_cu_subset); CL16
                                 operands read by the weight-grad only;
                                 6: LSTM layer GEMMs (se_gemm, se_colsum);
                                 5: prepared data-grad weight images (se_conv2d_prep_data_weights);
                                 4: SE_DTYPE storage types (CBN), first-block fused backward, se_resample */

enum {
  SE_OK = 0,
  SE_E_ARG = -1,          /* null pointer / negative size / bad flag          */
  SE_E_SHAPE = -2,        /* inconsistent shapes (e.g. reflect pad > length)  */
  SE_E_UNSUPPORTED = -3,  /* valid but not implemented (e.g. nfft radix)      */
  SE_E_LAUNCH = -4,       /* hipGetLastError() after a launch                 */
  SE_E_WORKSPACE = -5     /* ws_bytes smaller than *_workspace_size()         */
};

int se_abi_version(void);
const char* se_strerror(int code);

/* Loader self-test: out[i] = 3*i + 1 for i < n (one tiny kernel). */
int se_probe(int* out, int n, void* stream);

/* ------------------------------------------------------------------------
 * ConvSTFT / ConviSTFT (models/conv_stft.py:7-116)
 *
 * Both are computed as packed real FFTs in LDS (two frames per complex FFT
 * of length nfft), NOT as the reference's DFT-basis conv1d; the results are
 * the same linear maps (conv_stft.py:7-26 builds the basis from rfft(eye(N))
 * and its pinv). nfft must factor into 2,3,4,5 and be <= 1024; win <= nfft.
 *
 * window : fp32 [win]  periodic Hann (scipy get_window(win_type, win)).
 * twiddle: fp32 [2*nfft] interleaved (cos(2*pi*k/nfft), -sin(2*pi*k/nfft)).
 * ------------------------------------------------------------------------ */

/* Number of frames produced for a length-L signal (conv_stft.py:54-56). */
int se_stft_num_frames(int L, int win, int hop, int nfft, int center);

/* ConvSTFT.forward (conv_stft.py:48-66).
 * x: [B, L]. center=1 reflect-pads nfft/2 on both sides (requires L > nfft/2).
 * mag_phase=0: out0 = spec [B, nfft+2, T] (rows 0..nfft/2 real, rest imag).
 * mag_phase=1: out0 = mags [B, nfft/2+1, T], out1 = phase (atan2(im, re)).
 * dtype (SE_DTYPE_*): storage type of x and the outputs (fp32 arithmetic);
 * window / twiddle stay fp32 (the module's kernel tables). */
int se_stft_fwd(const void* x, void* out0, void* out1, int B, int L, int win,
                int hop, int nfft, int center, int mag_phase,
                const float* window, const float* twiddle, int dtype, void* stream);

/* ConviSTFT.forward (conv_stft.py:89-116) for a complex spec [B, nfft+2, T]:
 * overlap-add of the pinv-basis frames divided by (OLA(window^2) + 1e-8),
 * out[b, s] = full[b, s + offset] for 0 <= s < out_len. */
int se_istft_fwd(const void* spec, void* out, int B, int T, int win, int hop,
                 int nfft, int offset, int out_len, const float* window,
                 const float* twiddle, int dtype, void* stream);

/* Adjoint of se_istft_fwd: gspec = d(out)/d(spec)^T gout. */
int se_istft_bwd(const void* gout, void* gspec, int B, int T, int win,
                 int hop, int nfft, int offset, int out_len,
                 const float* window, const float* twiddle, int dtype, void* stream);

/* ------------------------------------------------------------------------
 * Complex (transposed) 2-D convolution as ONE fused implicit GEMM
 * (complex_nn.py:52-91). The four real convs of the reference
 *   re = Wr*xr - Wi*xi ,  im = Wi*xr + Wr*xi
 * become a single contraction against the block weight
 *   conv : [[Wr, -Wi], [Wi, Wr]]  in (Cout, Cin) layout
 *   convT: [[Wr,  Wi], [-Wi, Wr]] in (Cin, Cout) layout
 * assembled in the workspace from the two nn.Conv2d / nn.ConvTranspose2d
 * weight tensors (real_conv.weight, imag_conv.weight). Transposed convs are
 * split into stride-phase classes so no MFMA work is spent on inserted zeros.
 * Arithmetic: fp32 in / fp32 accumulate; the MFMA form is chosen by
 * se_conv2d_desc.math (below).
 * ------------------------------------------------------------------------ */
typedef struct se_conv2d_desc {
  int batch;
  int in_channels;    /* real channel count (2 x complex channels)          */
  int in_h, in_w;
  int out_channels;   /* real channel count (2 x complex channels)          */
  int kernel_h, kernel_w;
  int stride_h, stride_w;
  int pad_h, pad_w;
  int dil_h, dil_w;
  int out_pad_h, out_pad_w; /* ConvTranspose2d output_padding              */
  int transposed;     /* 0: ComplexConv2d, 1: ComplexConvTranspose2d         */
  int complex_weights;/* 1: (wr, wi) pair; 0: plain real conv, weight in wr  */
  int pad_h_end, pad_w_end; /* bottom / right padding; -1 = same as pad_h /
                       * pad_w (symmetric, nn.Conv2d). Asymmetric padding
                       * folds a zero pad of the input (e.g. FRCRN's causal
                       * F.pad(x, (1, 0)) before each encoder conv,
                       * frcrn.py:28-30) into the gather at no cost.          */
  int math;           /* SE_MATH_F32 (0): fp32 operands on v_mfma_f32_32x32x2_f32
                       * (exact fp32 products). SE_MATH_BF16X3 (1): each fp32
                       * operand split as hi + lo bf16, a*b ~ ah*bh + ah*bl +
                       * al*bh on v_mfma_f32_32x32x16_bf16, fp32 accumulate
                       * (<= ~2^-15 relative per product; fp32 in / fp32 out).
                       * SE_MATH_BF16X6 (2): three-way split h + m + l, six
                       * terms (hh, hm, mh, hl, lh, mm): fp32-class products;
                       * gather passes only (weight-grad runs SE_MATH_F32).
                       * SE_MATH_BF16 (3): operands rounded to bf16, one MFMA
                       * term, fp32 accumulate and storage (the arithmetic of a
                       * bf16 autocast conv; BASELINE configs 2/3).
                       * SE_MATH_F16X3 (4): scaled split-fp16. Each operand is
                       * multiplied by a power of two s (per tensor, from its
                       * max |.|: max|x| * s < 2^14) and split as hi + lo fp16
                       * (both round-to-nearest), a*b ~ ah*bh + ah*bl + al*bh on
                       * v_mfma_f32_32x32x16_f16, fp32 accumulate, the result
                       * multiplied back by 1/(s_a s_b) (exact). Per-product error
                       * <= ~2^-21 relative plus ~2^-38 max|a| |b| for elements
                       * below 2^-17 max|a|: fp32-class (tests/test_gpu_conv_x3.py
                       * asserts each pass at or below the SE_MATH_F32 path's
                       * error vs fp64) at the cost of bf16x3.
                       * Shapes the split kernels do not cover run SE_MATH_F32. */
  /* SE_MATH_F16X3 only: device pointers to ONE fp32 upper bound of max |.| of
   * the conv input x (for the joined entry points: over x and s) and of dy.
   * The bound may exceed the true maximum by up to ~2^10 without measurable
   * loss; it must not be below it. NULL = the call computes it (one extra read
   * of the tensor). Producers that already pass over the tensor (ComplexBN's
   * apply, se_amax) fill it for free. */
  const float* x_amax;
  const float* dy_amax;
  /* SE_MATH_F16X3 only, optional: device fp32 [1] holding an upper bound of
   * max |w| over the real and imaginary weights (se_amax_weights). The forward
   * and data-grad passes of one conv call share it (the weights do not change
   * between them); NULL = the pass computes it itself (two reductions). */
  const float* w_amax;
  /* ABI 4: SE_DTYPE_* storage of x, y, dy, dx, the weights, the biases and their
   * gradients. 16-bit storage (the reference's model.to(bfloat16) / .half()
   * runs) reads and writes those tensors as they are and computes with the
   * one-term MFMA of its own format, whose operands are then exact: bf16 needs
   * math SE_MATH_BF16, fp16 needs SE_MATH_F16 (SE_E_UNSUPPORTED otherwise, and for
   * the joined forms and the fp32-only small weight-grad shapes, before any
   * launch). fp32 storage takes any math. */
  int dtype;
  /* ABI 5, se_conv2d_bwd_data / se_conv2d_bwd_data_joined only, optional: the
   * pass's weight image (the per-class GEMM weight tiles and tap tables) already
   * built by se_conv2d_prep_data_weights from the same weights with a desc equal
   * in shape, math, dtype and w_amax. The pass then reads it instead of building
   * it in ws. A training step makes it in the forward, where the small prep
   * launch runs beside nothing, instead of in the backward, where it waits for CU
   * slots behind the side stream's weight-grad GEMMs. NULL = build it in ws. */
  const void* data_weights;
  /* ABI 8, the *_joined entry points only: the order of the joined input's channel
   * chunks. 0: complex_concat([x, s]) = [x_re, s_re, x_im, s_im] (FRCRN / DCCRN,
   * complex_nn.py:4-16), x_w >= in_w (x's extra columns cropped). 1: torch.cat([x, s])
   * = [x_re, x_im, s_re, s_im] (DCUNet's decoder, _1903_03107_dcunet.py:89-93),
   * x_w <= in_w (x zero-padded to the skip's grid, F.pad). x_h <= in_h either way. */
  int join_cat;
} se_conv2d_desc;

/* Bytes of the data-grad weight image of d (0 on an invalid desc). */
size_t se_conv2d_data_weights_size(const se_conv2d_desc* d);
/* Builds the data-grad weight image of (wr, wi) for d into img (see
 * se_conv2d_desc.data_weights). SE_MATH_F16X3 bakes the w_amax bound into the
 * image: d->w_amax must be set (SE_E_ARG otherwise) and the data pass must
 * pass the same bound. Replaces nothing in the reference (its conv re-reads the
 * module weights in each pass, complex_nn.py:52-65). */
int se_conv2d_prep_data_weights(const se_conv2d_desc* d, const float* wr, const float* wi, void* img,
                                size_t img_bytes, void* stream);

/* SE_MATH_F16 (5): operands rounded to fp16 (exact for fp16 storage), one MFMA
 * term on v_mfma_f32_32x32x16_f16, fp32 accumulate, no scaling (the reference's
 * model.half() conv). */
enum { SE_MATH_F32 = 0, SE_MATH_BF16X3 = 1, SE_MATH_BF16X6 = 2, SE_MATH_BF16 = 3,
       SE_MATH_F16X3 = 4, SE_MATH_F16 = 5 };

/* Storage types of the activation tensors an entry point reads and writes
 * (the reference's model.to(bfloat16) / model.half() runs, BASELINE configs
 * 2, 3, 5). Entry points without a dtype argument take fp32. */
enum { SE_DTYPE_F32 = 0, SE_DTYPE_BF16 = 1, SE_DTYPE_F16 = 2 };

/* amax[0] = max(amax[0], max_i |x[i]|) over n elements (atomic; zero amax[0]
 * first for a fresh maximum). The scale source of SE_MATH_F16X3. */
int se_amax(const float* x, long long n, float* amax, void* stream);
/* ABI 10: amax[0] = max_i |x[i]| (the slot zeroed by the call itself). */
int se_amax_init(const float* x, long long n, float* amax, void* stream);

/* max(max |wr|, max |wi|) of a conv's weights (wi may be NULL) written to
 * *amax by one single-workgroup launch (no zeroing, no atomics): the
 * se_conv2d_desc.w_amax of an SE_MATH_F16X3 conv call. */
int se_amax_weights(const float* wr, long long n, const float* wi, float* amax, void* stream);

/* Output spatial size (nn.Conv2d / nn.ConvTranspose2d formulas). */
int se_conv2d_out_shape(const se_conv2d_desc* d, int* out_h, int* out_w);

/* Workspace bytes needed by each of the calls below for this descriptor. */
size_t se_conv2d_workspace_size(const se_conv2d_desc* d);

/* y = conv(x) (+ bias). x: [B, Cin, Hi, Wi]; y: [B, Cout, Ho, Wo].
 * wr, wi: [Cout/2, Cin/2, kh, kw] (conv) or [Cin/2, Cout/2, kh, kw] (convT);
 * br, bi: [Cout/2] or NULL. Real mode: wr = full weight, br = full bias.   */
int se_conv2d_fwd(const se_conv2d_desc* d, const float* x, const float* wr,
                  const float* wi, const float* br, const float* bi, float* y,
                  void* ws, size_t ws_bytes, void* stream);

/* dx = d(y)/d(x)^T dy. */
int se_conv2d_bwd_data(const se_conv2d_desc* d, const float* dy,
                       const float* wr, const float* wi, float* dx, void* ws,
                       size_t ws_bytes, void* stream);

/* dwr, dwi (same shapes as wr, wi; OVERWRITTEN) and, if non-NULL, dbr, dbi. */
int se_conv2d_bwd_weight(const se_conv2d_desc* d, const float* x,
                         const float* dy, float* dwr, float* dwi, float* dbr,
                         float* dbi, void* ws, size_t ws_bytes, void* stream);

/* Decoder skip join folded into the conv GEMMs (frcrn.py:93-101: trim /
 * pad the decoder state x, complex_concat([x, s]), ConvTransposeBlock). The
 * conv input is the joined tensor [B, in_channels, in_h, in_w] with channel
 * chunks [x_re, s_re, x_im, s_im] of in_channels/4 each (d->join_cat = 1: [x_re,
 * x_im, s_re, s_im], torch.cat, DCUNet's decoder); it is never written.
 * s: [B, in_channels/2, in_h, in_w] (the CCBAM output); x: [B, in_channels/2,
 * x_h, x_w] with x_h <= in_h (missing rows read as zeros, F.pad(x, (0,0,0,1)))
 * and x_w >= in_w (extra columns unread, x[..., :-1]); with join_cat, x_w <= in_w
 * (missing columns read as zeros). Complex weights only, in_channels/4 a multiple
 * of 32. 16-bit storage (d->dtype) takes the one-term math of its format.
 * Returns SE_E_UNSUPPORTED when the math mode or shape has no joined kernel (the
 * split-bf16 / bf16 / f16 tap-uniform GEMMs have one; the weight-grad only for
 * transposed convs): the caller then materialises the join (se_complex_join, or a
 * concatenation for join_cat) and uses the plain entry points. */
int se_conv2d_fwd_joined(const se_conv2d_desc* d, const float* x, int x_h, int x_w,
                         const float* s, const float* wr, const float* wi,
                         const float* br, const float* bi, float* y, void* ws,
                         size_t ws_bytes, void* stream);
/* gx [B, in_channels/2, x_h, x_w] (zeros in the cropped columns and no
 * contribution from the padded rows / columns) and gs [B, in_channels/2, in_h, in_w]. */
int se_conv2d_bwd_data_joined(const se_conv2d_desc* d, const float* dy, const float* wr,
                              const float* wi, float* gx, int x_h, int x_w, float* gs,
                              void* ws, size_t ws_bytes, void* stream);
int se_conv2d_bwd_weight_joined(const se_conv2d_desc* d, const float* x, int x_h, int x_w,
                                const float* s, const float* dy, float* dwr, float* dwi,
                                float* dbr, float* dbi, void* ws, size_t ws_bytes,
                                void* stream);

/* ------------------------------------------------------------------------
 * ComplexBatchNorm2d (complex_nn.py:148-329) with optional fused
 * LeakyReLU / ReLU (frcrn.py:22,34; ccbam.py:12,15).
 * x, y: [B, C, H, W], C = 2*Cc. Per complex channel: mean (Mr, Mi), biased
 * covariance (Vrr, Vri, Vii) + eps, U = V^-1/2 by the closed 2x2 form
 * (complex_nn.py:288-297), Z = W U with symmetric W, y = Z (x - M) + B.
 * Moments are accumulated in fp64 (one pass over x).
 *
 * params : host array of 5 device pointers Wrr, Wri, Wii, Br, Bi, each fp32
 *          [Cc] (the module's nn.Parameters), or NULL when affine=False.
 * running: host array of 5 device pointers RMr, RMi, RVrr, RVri, RVii, or
 *          NULL when track_running_stats=False; updated in place in training.
 * nbt    : device int64 num_batches_tracked (NULL if not tracking).
 * save   : device fp32 [SE_CBN_SAVE_FLOATS*Cc] per-channel state for se_cbn_bwd.
 * act    : 0 none, 1 LeakyReLU(slope), 2 ReLU (applied after the affine).
 * training: 1 = batch statistics (+ running update when running != NULL),
 *          0 = running statistics.
 * momentum < 0 means "None" (cumulative average, complex_nn.py:223-224).
 * y_amax : device fp32 [1] or NULL. Training only: receives an upper bound of
 *          max |y| (from the moments pass's per-channel extrema, no extra
 *          pass), the se_conv2d_desc.x_amax of a SE_MATH_F16X3 consumer.
 * prelu_w: NULL, or (with act = 1) the device weight of an nn.PReLU() with one
 *          parameter applied after the norm (DCCRN, dccrn.py:21,45): LeakyReLU
 *          with the slope read on the device. The backward writes its gradient
 *          to dprelu_w (one element, overwritten).
 * dtype  : SE_DTYPE_F32 / BF16 / F16, the storage type of x, y, gy, gy2, dx AND
 *          of params / dparams / running / prelu_w (a model.to(bfloat16) /
 *          .half() module keeps all of them in its dtype). Arithmetic is fp32
 *          (moments fp64); stores round to nearest even. save stays fp32.
 * ------------------------------------------------------------------------ */
#define SE_CBN_SAVE_FLOATS 20
size_t se_cbn_workspace_size(int B, int C, int HW);

int se_cbn_fwd(const void* x, void* y, int B, int C, int HW,
               const void* const* params, void* const* running,
               int64_t* nbt, float* save, int training, float eps,
               float momentum, int act, float slope, float* y_amax,
               const void* prelu_w, int dtype, void* ws, size_t ws_bytes,
               void* stream);

/* Backward. gy = dL/dy (after the activation), x = forward input. y (the
 * forward output) is NOT read and may be NULL: the activation derivative is
 * taken from the pre-activation Z(x - M) + B recomputed from x and `save`.
 * dx is overwritten. dparams: host array of 5 device pointers dWrr, dWri,
 * dWii, dBr, dBi (overwritten), or NULL. dx_amax: device fp32 [1] or NULL;
 * training only: an upper bound of max |dx| (the se_conv2d_desc.dy_amax of the
 * producing conv's SE_MATH_F16X3 backward). */
int se_cbn_bwd(const void* gy, const void* y, const void* x, void* dx,
               int B, int C, int HW, const void* const* params,
               const float* save, void* const* dparams, int training,
               int act, float slope, float* dx_amax, const void* prelu_w, void* dprelu_w,
               int dtype, void* ws, size_t ws_bytes, void* stream);

/* Backward of a forked output: y feeds two consumers (FRCRN's encoder block
 * output is the next encoder conv's input and the decoder skip, frcrn.py:70-75,
 * 93-95), so dL/dy = gy + gy2. The sum is formed on the fly in both passes;
 * autograd's separate gradient-accumulation add (2 reads + 1 write of an
 * activation-sized tensor) is never run. gy2 must not be NULL. Otherwise as
 * se_cbn_bwd. */
int se_cbn_bwd2(const void* gy, const void* gy2, const void* x, void* dx,
                int B, int C, int HW, const void* const* params,
                const float* save, void* const* dparams, int training,
                int act, float slope, float* dx_amax, const void* prelu_w, void* dprelu_w,
                int dtype, void* ws, size_t ws_bytes, void* stream);

/* ABI 11. Backward of a forked output whose second consumer is FRCRN's CCBAM skip gate
 * (frcrn.py:70-75, 93-95; ccbam.py:28-106): dL/dy = gy + the gate's input gradient, formed
 * on the fly in both passes from the gate's parts instead of being written by a separate
 * pass (se_ccbam_bwd_dx) and read back. At (b, channel ch = h C/2 + cc, position i):
 *   gy2 = (g + dP[b, 2h, i] / (C/2) + [idx[b, h, i] == cc] dP[b, 2h + 1, i]) ca[b, ch]
 *         + dmean[b, ch] / HW + [amax[b, ch] == i] dmax[b, ch]
 * with g_gate [B, C, HW] the gate's output gradient and dP / idx / ca / dmean / dmax / amax
 * as se_ccbam_bwd_dx takes them. fp32; LeakyReLU / ReLU / none (no PReLU). Otherwise as
 * se_cbn_bwd (workspace se_cbn_workspace_size). Replaces se_ccbam_bwd_dx + se_cbn_bwd2. */
int se_cbn_bwd_ccbam(const float* gy, const float* g_gate, const float* dP, const short* idx,
                     const float* ca, const float* dmean, const float* dmax, const int* amax,
                     const float* x, float* dx, int B, int C, int HW, const float* const* params,
                     const float* save, float* const* dparams, int training, int act, float slope,
                     float* dx_amax, void* ws, size_t ws_bytes, void* stream);

/* Output head fused into the last ComplexBatchNorm2d (frcrn.py:115, 140-144):
 * FRCRN's final_conv = nn.Conv2d(C, 2, kernel_size=(1, 2), bias=False) applied
 * to y = act(CBN(x)) of the last decoder block, whose only consumer it is.
 * se_cbn_head_fwd writes out [B, 2, H, W-1] = final_conv(y) without writing y
 * (replaces se_cbn_fwd + the real conv's forward: 2 activation-sized passes
 * fewer); se_cbn_head_bwd takes gout = dL/dout and forms dL/dy inside both
 * backward passes, writes dx as se_cbn_bwd, and the head's weight gradient
 * dw_head [2, C, 1, 2] (overwritten) from y recomputed in the moments pass
 * (replaces the conv's data-grad and weight-grad and se_cbn_bwd's gy reads).
 * x: [B, C, H, W]; w_head: [2, C, 1, 2] fp32. out_channels must be 2 and
 * kernel_w 2 (SE_E_UNSUPPORTED otherwise). Other arguments as se_cbn_fwd /
 * se_cbn_bwd; the workspace is se_cbn_head_workspace_size(B, C, H * W) bytes
 * for both. */
size_t se_cbn_head_workspace_size(int B, int C, int HW);

int se_cbn_head_fwd(const float* x, float* out, int B, int C, int H, int W,
                    const float* const* params, float* const* running, int64_t* nbt,
                    float* save, int training, float eps, float momentum, int act,
                    float slope, const float* w_head, int out_channels, int kernel_w,
                    void* ws, size_t ws_bytes, void* stream);

int se_cbn_head_bwd(const float* gout, const float* x, float* dx, int B, int C, int H, int W,
                    const float* const* params, const float* save, float* const* dparams,
                    const float* w_head, float* dw_head, int out_channels, int kernel_w,
                    int training, int act, float slope, float* dx_amax, void* ws,
                    size_t ws_bytes, void* stream);

/* First block (conv -> ComplexBatchNorm2d [+ act]) whose conv input x0 needs no
 * gradient: a model's first, data-fed conv (FRCRN's encoder layer 0,
 * frcrn.py:28-34, 62-76). se_cbn_bwd_first_conv is se_cbn_bwd / se_cbn_bwd2
 * (gy2 may be NULL) with the conv's weight gradient accumulated inside the apply
 * pass from the dL/dy0 it computes, in exact fp32 products: dL/dy0 (the conv's
 * dy, an activation-sized tensor) is never written, and the conv's separate
 * weight-grad pass (which reads it back) is replaced. Replaces the conv's
 * se_conv2d_bwd_weight and the CBN's dx write. The conv is complex, bias-free,
 * with cin = in_channels / 2 complex input channels; supported: cin = 1, kernel
 * (5, 2) (SE_E_UNSUPPORTED otherwise). Paddings are the begin paddings (an
 * asymmetric pad is folded in as se_conv2d_desc). x: [B, C, H, W] (the conv
 * output = CBN input); dwr / dwi: [C/2, cin, kh, kw] (overwritten). Workspace:
 * se_cbn_first_conv_workspace_size bytes. */
typedef struct {
  const float* x0;        /* conv input [B, 2*cin, in_h, in_w] */
  int cin, in_h, in_w;
  int kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w;
  float* dwr;
  float* dwi;
} se_first_conv;
size_t se_cbn_first_conv_workspace_size(int B, int C, int HW, int cin, int kh, int kw);
int se_cbn_bwd_first_conv(const float* gy, const float* gy2, const float* x, int B, int C, int H, int W,
                          const float* const* params, const float* save, float* const* dparams,
                          int training, int act, float slope, const se_first_conv* fc, void* ws,
                          size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * LSTM recurrence (torch.nn.LSTM as used by ComplexLSTM, complex_nn.py:115-145)
 *
 * L independent single-layer LSTMs with hidden size H in {64, 128}, batch B
 * (even), T steps, h0 = c0 = 0, gate order i, f, g, o. The input projection
 * xproj = X W_ih^T + b_ih + b_hh (row (l, b*T + t) at
 * xproj + l*x_lstm_stride + (b*T + t)*x_row_stride, 4H wide) and every
 * weight gradient are plain GEMMs left to the caller. Bit l of rev_mask runs
 * LSTM l right-to-left (the reverse half of a bidirectional layer).
 *
 * zero  : device fp32 [H] of zeros (h_{-1}; read with scalar loads)
 * h, c  : fp32 [L][B][T][H]   outputs (h) and cell states (saved for bwd)
 * gates : fp32 [L][B][T][4H]  post-activation gates (saved for bwd)
 * dy    : fp32 [L][B][T][H]   dLoss/dh
 * dgates: fp32 [L][B][T][4H]  dLoss/d(pre-activation gates); then
 *         dW_ih = dgates^T X, dW_hh = dgates^T h_prev, db = sum dgates,
 *         dX = dgates W_ih.
 * ------------------------------------------------------------------------ */
int se_lstm_supported(int hidden);
int se_lstm_fwd(const float* xproj, long long x_lstm_stride, int x_row_stride,
                const float* w_hh, const float* zero, float* h, float* c, float* gates, int L,
                int B, int T, int H, unsigned rev_mask, void* stream);
int se_lstm_bwd(const float* dy, const float* w_hh, const float* gates,
                const float* c, float* dgates, int L, int B, int T, int H,
                unsigned rev_mask, void* stream);

/* The LSTM layer GEMMs (ABI 6; replace the torch.addmm / bmm calls that the
 * nn.LSTM input projection and weight / input gradients ran on rocBLAS) and,
 * ABI 10, every nn.Linear / ComplexLinear of the models (complex_nn.py:93-113,
 * DCCRN's LSTMBlock dccrn.py:71-86, CARN's head carn.py:133,157-159):
 *   C[b](m, n) = sum_k A(b, m, k) B(b, k, n) (+ bias0 + bias1)
 *   A(b, m, k) = A[b stride_a + m lda + k] (a_mcontig 0) | A[b stride_a + k lda + m] (1)
 *   B(b, k, n) = B[b stride_b + n ldb + k] (b_ncontig 0) | B[b stride_b + k ldb + n] (1)
 *   C[b](m, n) at C[b stride_c + m ldc + n]; sum_batches = 1: one C, the sum of
 *   the batch products (in batch order, inside the accumulation).
 *   bias (bias0[b stride_bias + i] + bias1[...]) with i = n (bias_rows 0) or m (1).
 * A(m, k) reads as 0 where k % kmask_period == kmask_phase (period 0: none).
 * dtype SE_DTYPE_F32: scaled split-fp16 (f16x3, as SE_MATH_F16X3) with per-tensor
 * power-of-two scales from amax_a / amax_b (device fp32 upper bounds of max |A|,
 * max |B|). SE_DTYPE_BF16 / _F16 (ABI 10): A, B, C and the biases in that format,
 * one-term MFMA of it (exact products, fp32 accumulation, C rounded once; amax
 * pointers unused). splits: split-K slabs (0: the library picks from the shape);
 * with more than one the workspace holds the fp32 slabs, added in split order.
 * se_colsum: out[l][g] = sum_r x[l][r][g] (the LSTM bias gradient; 64 row chunks,
 * each in row order, then the chunks in order) and, if amax is not NULL, max |x|
 * into *amax (the scale source of the weight-gradient GEMMs over x).
 * se_bias_grad (ABI 10): out[g] = sum_l sum_r x[l sl + r sr + g sg] in fp32, rounded
 * to dtype once (a Linear's bias gradient over any layout of dy; chunked like
 * se_colsum when sg = 1, one wave per g over contiguous rows when sr = 1). */
typedef struct se_gemm_desc {
  int M, N, K;
  int batches, sum_batches;
  int a_mcontig, b_ncontig;
  int lda, ldb, ldc;
  long long stride_a, stride_b, stride_c, stride_bias;
  int kmask_period, kmask_phase;
  int splits;
  int dtype;       /* ABI 10: SE_DTYPE_* of A, B, C and the biases */
  int bias_rows;   /* ABI 10: 1 = bias indexed by m */
} se_gemm_desc;
size_t se_gemm_workspace_size(const se_gemm_desc* d);
int se_gemm(const se_gemm_desc* d, const void* A, const void* B, void* C, const void* bias0,
            const void* bias1, const float* amax_a, const float* amax_b, void* ws, size_t ws_bytes,
            void* stream);
size_t se_colsum_workspace_size(int L, long long R, int G);
int se_colsum(const float* x, int L, long long R, int G, float* out, float* amax, void* ws, size_t ws_bytes,
              void* stream);
size_t se_bias_grad_workspace_size(int L, long long R, int G);
int se_bias_grad(const void* x, int L, long long R, int G, long long sl, long long sr, long long sg, int dtype,
                 void* out, void* ws, size_t ws_bytes, void* stream);

/* Strided copy with a storage-type conversion (ABI 10): dst[i] = (dst type) src[i]
 * over an ndim <= SE_COPY_MAX_DIMS index space (host arrays sizes / src_strides /
 * dst_strides, in elements). The layout changes and casts of the models' glue
 * (.contiguous() of a transposed or sliced view, .float() / .to(dtype), the
 * re / im stacking of ComplexLSTM, the per-layer LSTM weight stacks) as one pass. */
#define SE_COPY_MAX_DIMS 5
int se_copy_strided(const void* src, int src_dtype, void* dst, int dst_dtype, int ndim, const long long* sizes,
                    const long long* src_strides, const long long* dst_strides, void* stream);

/* ComplexLSTM's output (complex_nn.py:134-142), ABI 10: from the stacked
 * recurrence h [2][2B][T][H] fp32 (LSTM 0 = real_lstm, 1 = imag_lstm; batch rows
 * [0, B) ran the real part, [B, 2B) the imaginary part; h_lstm_stride between the
 * LSTMs) -> out[b, t, k] (dtype): re = real(re) - imag(im) for k < H,
 * im = imag(re) + real(im) for k >= H, at out + b out_batch_stride + t out_row_stride +
 * k out_feature_stride (feature stride 1: [B, T, 2H] rows; row stride 1: the [B, 2H, T]
 * layout a conv stack reads next). The backward scatters gout (same stride convention)
 * into dh [2][2B][T][H] fp32 (every element written). */
int se_complex_lstm_combine_fwd(const float* h, long long h_lstm_stride, int B, int T, int H, void* out,
                                long long out_batch_stride, long long out_row_stride, long long out_feature_stride,
                                int dtype, void* stream);
int se_complex_lstm_combine_bwd(const void* gout, long long g_batch_stride, long long g_row_stride,
                                long long g_feature_stride, int B, int T, int H, int dtype, float* dh,
                                long long dh_lstm_stride, void* stream);

/* Wide hidden sizes, H in {256, 512, 1024} (CARN's nn.LSTM(512), models/
 * _2104_05267_carn.py:132; CRN's nn.LSTM(1024), models/_1809_01405_crn.py:90;
 * replaces the MIOpen per-step kernels behind them): same arguments, layouts
 * and results as se_lstm_fwd / se_lstm_bwd (no zero row; any B). W_hh is
 * spread over a group of H/U workgroups (U = 32, 16 at H = 1024), each holding
 * the gate rows (fwd) / columns (bwd) of U hidden units in registers; the
 * group exchanges h_t / dgates_t through the outputs every step.
 * sync  : device int[se_lstm_wide_sync_ints()] scratch (zeroed by the call)
 * status: device int; set non-zero if a group barrier timed out (the outputs
 *         are then NaN from that step on); never cleared by the library.
 * A batch whose groups cannot all be resident at once runs as consecutive
 * launches over slices of it; SE_E_UNSUPPORTED only when L LSTMs of 8
 * sequences do not fit (L * H / U > number of CUs). */
int se_lstm_wide_supported(int hidden);
int se_lstm_wide_sync_ints(void);
int se_lstm_wide_fwd(const float* xproj, long long x_lstm_stride, int x_row_stride,
                     const float* w_hh, float* h, float* c, float* gates, int L, int B,
                     int T, int H, unsigned rev_mask, int* sync, int* status, void* stream);
int se_lstm_wide_bwd(const float* dy, const float* w_hh, const float* gates,
                     const float* c, float* dgates, int L, int B, int T, int H,
                     unsigned rev_mask, int* sync, int* status, void* stream);

/* ------------------------------------------------------------------------
 * Real BatchNorm2d + activation (CARN / GCARN ConvBlock: BatchNorm2d + PReLU,
 * models/_2104_05267_carn.py:30-56; CRN ConvBlock: BatchNorm2d + ELU,
 * models/_1809_01405_crn.py:9-45), fwd (training: batch statistics + running
 * stat update with a float momentum; eval: running stats) and bwd.
 * x     : B*C planes of HW contiguous floats, plane (b, c) at
 *         x + (b*C + c)*x_plane_stride (a row-cropped view qualifies)
 * y, gy, dx : contiguous [B][C][HW]
 * weight, bias : [C] or NULL (affine=False); dweight / dbias likewise
 * act   : 0 none, 1 PReLU (act_param [1] or [C] when act_per_channel),
 *         2 ELU(elu_alpha); dact_param: the PReLU weight gradient
 * save  : device fp32 [2C] = {mean, invstd} used, written by se_bn_fwd
 * dtype : SE_DTYPE_* of x, y, gy, dx AND weight, bias, running stats, act_param and
 *         their gradients (a model.half() / .to(bfloat16) module); fp32 arithmetic
 * ws    : se_bn_workspace_size(B, C) bytes (training fwd and every bwd)
 * ------------------------------------------------------------------------ */
size_t se_bn_workspace_size(int B, int C);
int se_bn_fwd(const void* x, long long x_plane_stride, int B, int C, int HW, const void* weight,
              const void* bias, void* running_mean, void* running_var, int training, float momentum,
              float eps, int act, const void* act_param, int act_per_channel, float elu_alpha, void* y,
              float* save, int dtype, void* ws, size_t ws_bytes, void* stream);
int se_bn_bwd(const void* gy, const void* x, long long x_plane_stride, int B, int C, int HW,
              const void* weight, const void* bias, const float* save, int training, int act,
              const void* act_param, int act_per_channel, float elu_alpha, void* dx, void* dweight,
              void* dbias, void* dact_param, int dtype, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Train-step glue (trainer.py:99-124, :210-221)
 *
 * SI-SNR loss (losses.py:62-84) of B estimates against B targets [B, lt]
 * with utils.py:111-121's pad / truncate folded in: estimate row b is
 * est + b*est_stride, le samples (zero past le, ignored past lt).
 * loss: device fp32 [1] = -mean_b 10 log10(signal / noise);
 * save: device scratch of se_sisnr_save_bytes(B), kept for se_sisnr_bwd;
 * grad_est: [B] rows of le (stride grad_stride) = grad_loss[0] * dloss/dest.
 *
 * Parameter update over a device table of slots (the concatenation of every
 * tensor; offset = prefix sum of numel, slots in offset order):
 * se_grad_sumsq   : sumsq[0] = sum of grad^2 (fp64, device; sumsq holds
 *                   SE_SUMSQ_DOUBLES doubles: [1..] are per-workgroup
 *                   partials, added in a fixed order: deterministic);
 * se_clip_grads   : grads *= min(max_norm / (sqrt(*sumsq) + 1e-6), 1)
 *                   (torch.nn.utils.clip_grad_norm_; total_norm -> [1] if set);
 * se_adamw_step   : torch.optim.AdamW (amsgrad off) at step `step` (>= 1).
 * ------------------------------------------------------------------------ */
#define SE_SUMSQ_DOUBLES 2049
typedef struct se_tensor_slot {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long numel;
  long long offset;
} se_tensor_slot;

/* FRCRN's complex-ratio mask (frcrn.py:140-152): h = final_conv output
 * [B, 2, half - 2, T] (half = nfft/2 + 1), spec = ConvSTFT output [B, 2*half, T];
 * est [B, 2*half, T] = pad(tanh(pad(h, top 1)) * spec[:, :, 1:], top 1), i.e.
 * est[b, c*half + k, t] = k < 2 ? 0 : tanh(h[b, c, k-2, t]) * spec[b, c*half + k, t].
 * se_mask_bwd: gh = gest * spec * (1 - tanh(h)^2) on rows k >= 2 (spec takes no
 * gradient). Replaces the pad / tanh / mul / pad / cat kernels of the reference. */
int se_mask_fwd(const float* h, const float* spec, int B, int half, int T, float* est, void* stream);
int se_mask_bwd(const float* gest, const float* h, const float* spec, int B, int half, int T, float* gh,
                void* stream);

/* The magnitude / phase masks (DCUNet, DCCRN), ABI 9. mode 0: DCUNet's
 * bounded_tanh (models/_1903_03107_dcunet.py:167-189, ph = n_ph + m_ph / m_mag); mode 1: DCCRN's
 * 'E' (models/_2008_00264_dccrn.py:194-207, m_ph = atan2(mi / m_mag, mr / m_mag), ph = n_ph + m_ph);
 * both gain = n_mag * tanh(m_mag), mag = sqrt(re^2 + im^2 + 1e-8), phase = atan2(im, re).
 * out [B, 2, F, T] = gain * (cos ph, sin ph). Mask (mr, mi) and noisy (nr, ni) planes: time
 * contiguous, the given batch / row strides in elements. dtype SE_DTYPE_*: every intermediate
 * rounded to it as the reference's tensors are. Replaces ~20 elementwise kernels. */
int se_polar_mask_fwd(const void* mr, const void* mi, long long m_batch_stride, long long m_row_stride,
                      const void* nr, const void* ni, long long n_batch_stride, long long n_row_stride, int B, int F,
                      int T, int mode, int dtype, int m_row0, void* out, void* stream);
/* Its backward for a training forward (ABI 9): g = dL/dout [B, 2, F, T] -> dm = (dL/dmr, dL/dmi);
 * the noisy planes take no gradient. fp32 arithmetic on the storage values (the forward's
 * intermediates recomputed), gradients rounded to dtype once.
 * ABI 10, m_row0: the mask's first m_row0 rows are zeros that are not stored (DCCRN's
 * F.pad(mask, (0, 0, 1, 0)), dccrn.py:172): mask row f >= m_row0 is read at stored row
 * f - m_row0. dm is [B, 2, F - m_row0, dm_T] (dm_T >= T; columns t >= T written as 0: the
 * frame the reference trims off the mask, dccrn.py:180-182), the gradient of the stored mask. */
int se_polar_mask_bwd(const void* g, const void* mr, const void* mi, long long m_batch_stride,
                      long long m_row_stride, const void* nr, const void* ni, long long n_batch_stride,
                      long long n_row_stride, int B, int F, int T, int mode, int dtype, int m_row0, int dm_T,
                      void* dm, void* stream);

/* ABI 10: dtype (SE_DTYPE_*) is the storage type of est, target, loss, grad_loss and
 * grad_est (a model.to(bfloat16) / .half() run); the sums stay fp64, the loss and the
 * gradient are rounded to dtype once. The slot tables' param / grad / exp_avg /
 * exp_avg_sq are all of the slot functions' dtype: 16-bit AdamW rounds each
 * intermediate to it where torch's foreach AdamW stores one (p *= 1 - lr wd;
 * m.lerp_(g, 1 - b1); v *= b2; v.addcmul_(g, g, 1 - b2); d = sqrt(v) / bc2_sqrt + eps in
 * three rounded steps; p.addcdiv_(m, d, -step_size)), and 16-bit clipping scales by
 * the coefficient rounded to dtype (torch multiplies by a dtype tensor). */
size_t se_sisnr_save_bytes(int B);
int se_sisnr_fwd(const void* est, int le, long long est_stride, const void* target, int lt, int B,
                 int zero_mean, float eps, void* loss, void* save, int dtype, void* stream);
int se_sisnr_bwd(const void* est, int le, long long est_stride, const void* target, int lt, int B,
                 int zero_mean, float eps, const void* save, const void* grad_loss, void* grad_est,
                 long long grad_stride, int dtype, void* stream);
int se_grad_sumsq(const se_tensor_slot* slots, int nslots, long long total, double* sumsq, int dtype, void* stream);
int se_clip_grads(const se_tensor_slot* slots, int nslots, long long total, const double* sumsq,
                  float max_norm, float* total_norm, int dtype, void* stream);
int se_adamw_step(const se_tensor_slot* slots, int nslots, long long total, double lr, double beta1,
                  double beta2, double eps, double weight_decay, long long step, int dtype, void* stream);

/* ------------------------------------------------------------------------
 * Complex CBAM skip attention (models/modules/ccbam.py:28-106), the passes
 * over the full skip tensor x [B, C, HW] (C even, <= 512; channels [0, C/2)
 * real, [C/2, C) imag). The shared MLP (ccbam.py:38-41) and the 4->2 k7
 * ComplexConv2d + CBN + ReLU (ccbam.py:65-71) run as their own modules on
 * the small pooled maps. Max-pool gradients go to the first maximal index
 * (AdaptiveMaxPool2d / torch.max(dim) semantics).
 *
 * channel_pool : mean, max, first argmax over HW per (b, c)   [B, C]
 * spatial_pool : pooled [B, 4, HW] = (mean_re, max_re, mean_im, max_im) of
 *                x*ca over each half's channels; idx int16 [B, 2, HW] = the
 *                argmax channel within the half (ccbam.py:73-83)
 * apply        : out = x*ca + sa[b, half(c)]                   (ccbam.py:98-105)
 * bwd_sa       : dsa [B, 2, HW] = per-half channel sums of gout
 * bwd_dca      : dca [B, C] = sum_hw gx1*x, gx1 = gout + dpooled_mean/(C/2)
 *                + [argmax] dpooled_max; needs se_ccbam_workspace_size bytes
 * bwd_dx       : dx = gx1*ca + dmean/HW + [hw == argmax_hw(b,c)] dmax
 * ------------------------------------------------------------------------ */
size_t se_ccbam_workspace_size(int B, int C, int HW);
int se_ccbam_channel_pool(const float* x, float* mean, float* mx, int* amax,
                          int B, int C, int HW, void* stream);
int se_ccbam_spatial_pool(const float* x, const float* ca, float* pooled,
                          short* idx, int B, int C, int HW, void* stream);
/* ABI 10: out_amax (or NULL) receives max |out| (the slot zeroed by the call). */
int se_ccbam_apply(const float* x, const float* ca, const float* sa, float* out,
                   int B, int C, int HW, float* out_amax, void* stream);
int se_ccbam_bwd_sa(const float* gout, float* dsa, int B, int C, int HW,
                    void* stream);
/* ABI 6: se_ccbam_bwd_sa with the spatial gate's sigmoid backward fused:
 * dz = (sum of gout over each half's channels) * (1 - sa) * sa, sa = sigmoid(z) the gate
 * [B, 2, HW]; bit-identical to se_ccbam_bwd_sa followed by torch's sigmoid_backward. */
int se_ccbam_bwd_sa_sigmoid(const float* gout, const float* sa, float* dz, int B, int C, int HW, void* stream);
int se_ccbam_bwd_dca(const float* gout, const float* x, const float* dpooled,
                     const short* idx, float* dca, int B, int C, int HW,
                     void* ws, size_t ws_bytes, void* stream);
int se_ccbam_bwd_dx(const float* gout, const float* dpooled, const short* idx,
                    const float* ca, const float* dmean, const float* dmax,
                    const int* amax, float* dx, int B, int C, int HW,
                    void* stream);

/* Channel-attention MLP (ccbam.py:28-63, ComplexLinear complex_nn.py:93-113):
 * ca [B, C] = sigmoid(f(mean) + f(max)), f = ComplexLinear(C, Hd, bias=False) ->
 * ReLU -> ComplexLinear(Hd, C, bias=False), each ComplexLinear a real_linear on the
 * first half of the features and an imag_linear on the second (no cross terms).
 * w1r / w1i: [Hd/2][C/2], w2r / w2i: [C/2][Hd/2] (the nn.Linear weights). hsave
 * [2B, Hd] (the ReLU outputs, avg rows then max rows) is written for the backward.
 * se_ccbam_mlp_bwd: from dca, dmean / dmax [B, C] and the four weight gradients
 * (overwritten; fp64 sums over the 2B rows). One workgroup each; needs
 * (B*C + 2*B*Hd) floats of LDS <= 64 KB (SE_E_UNSUPPORTED otherwise). */
int se_ccbam_mlp_fwd(const float* mean, const float* mx, const float* w1r, const float* w1i,
                     const float* w2r, const float* w2i, int B, int C, int Hd, float* ca,
                     float* hsave, void* stream);
int se_ccbam_mlp_bwd(const float* dca, const float* ca, const float* mean, const float* mx,
                     const float* hsave, const float* w1r, const float* w1i, const float* w2r,
                     const float* w2i, int B, int C, int Hd, float* dmean, float* dmx,
                     float* dw1r, float* dw1i, float* dw2r, float* dw2i, void* stream);

/* ------------------------------------------------------------------------
 * CARN / GCARN glue (models/_2104_05267_carn.py), ABI 10. dtype SE_DTYPE_* of
 * every tensor; fp32 arithmetic, rounded to dtype where the reference's tensors are.
 *
 * se_carn_mask_fwd (carn.py:161-168): m [B, 2, half, T] (the head Linear's output,
 * batch stride m_batch_stride, planes contiguous), spec [B, 2 half, T] (the
 * ConvSTFT output: rows [0, half) real, [half, 2 half) imag) ->
 *   est[b, f]        = mr nr - mi ni
 *   est[b, half + f] = mr ni - mi nr        (the reference's sign, as written)
 * se_carn_mask_bwd: gest -> dm [B, 2, half, T] and, if dspec is not NULL, dspec.
 * se_add_sigmoid_fwd: y = sigmoid(a + b) (Attention, carn.py:70-72); se_sigmoid_bwd:
 * dz = g (1 - y) y (torch's sigmoid_backward), the gradient of both a and b.
 * se_gate_cat_fwd: out [B, 2C, HW] = cat(sigmoid(c) * skip, skip) (carn.py:74-76 and
 * the decoder's torch.cat, :112-113); se_gate_cat_bwd: dc, dskip (both halves).
 * se_glu_fwd / _bwd: y = a * sigmoid(b) (ConvGLU / DeConvGLU, carn.py:9-27).
 * se_clamp_fwd / _bwd: y = clamp(x, lo, hi); dx = g where lo <= x <= hi else 0
 * (the models' torch.clamp_(wav, -1, 1), e.g. carn.py:170, frcrn.py:154).
 * ------------------------------------------------------------------------ */
int se_carn_mask_fwd(const void* m, long long m_batch_stride, const void* spec, int B, int half, int T, int dtype,
                     void* est, void* stream);
int se_carn_mask_bwd(const void* gest, const void* m, long long m_batch_stride, const void* spec, int B, int half,
                     int T, int dtype, void* dm, void* dspec, void* stream);
int se_add_sigmoid_fwd(const void* a, const void* b, void* y, long long n, int dtype, void* stream);
/* y = sigmoid(x) = 1 / (1 + exp(-x)) (accurate expf; e.g. CCBAM's spatial gate, ccbam.py:86). */
int se_sigmoid_fwd(const void* x, void* y, long long n, int dtype, void* stream);
int se_sigmoid_bwd(const void* g, const void* y, void* dz, long long n, int dtype, void* stream);
int se_gate_cat_fwd(const void* c, const void* skip, void* out, int B, int C, long long HW, int dtype, void* stream);
int se_gate_cat_bwd(const void* gout, const void* c, const void* skip, void* dc, void* dskip, int B, int C,
                    long long HW, int dtype, void* stream);
int se_glu_fwd(const void* a, const void* b, void* y, long long n, int dtype, void* stream);
int se_glu_bwd(const void* g, const void* a, const void* b, void* da, void* db, long long n, int dtype,
               void* stream);
int se_clamp_fwd(const void* x, void* y, long long n, float lo, float hi, int dtype, void* stream);
int se_clamp_bwd(const void* g, const void* x, void* dx, long long n, float lo, float hi, int dtype, void* stream);

/* Long-form chunking (sehip/longform.py, BASELINE config 5), ABI 10:
 * se_chunk_split: out [n, chunk] = x[i hop + s] (0 at or past L);
 * se_chunk_overlap_add: y [n, width] (the enhanced chunks, 0 past width) ->
 * out [length]: each chunk weighted by a linear cross-fade over its overlaps
 * (fade in (j + 0.5) / overlap on its first `overlap` samples unless first, fade out
 * 1 - that on its last unless last), summed in chunk order, rounded to dtype at
 * each step as the reference-side loop does. */
int se_chunk_split(const void* x, long long L, int n, int chunk, int hop, int dtype, void* out, void* stream);
int se_chunk_overlap_add(const void* y, int n, int width, int chunk, int overlap, long long length, int dtype,
                         void* out, void* stream);

/* ------------------------------------------------------------------------
 * Decoder skip join (models/_2206_07293_frcrn.py:93-100 + complex_concat,
 * complex_nn.py:4-16): out = [x_re, s_re, x_im, s_im] on channels, with x
 * [B, Cx, Fx, Tx] cropped / zero-padded at the end of each spatial dim to
 * s's [F, T] (x[..., :-1] and F.pad(x, (0, 0, 0, 1)) in the reference).
 * out: [B, Cx + Cs, F, T]. Backward writes gx over x's own grid (zeros where
 * x was cropped) and gs. dtype (SE_DTYPE_*, ABI 4): storage type of all the
 * tensors (a bf16 / fp16 model's decoder, e.g. DCCRN's, dccrn.py:116-120).
 * ------------------------------------------------------------------------ */
int se_complex_join(const void* x, int Cx, int Fx, int Tx, const void* s,
                    int Cs, int F, int T, void* out, int B, int dtype, void* stream);
int se_complex_join_bwd(const void* gout, void* gx, int Cx, int Fx, int Tx,
                        void* gs, int Cs, int F, int T, int B, int dtype, void* stream);

/* ------------------------------------------------------------------------
 * Data path: the reference mixes and crops on the host
 * (mix_audio.py:87-123, audio_dataloader.py:29-50); here the per-sample work
 * runs on the device and the host keeps only the random draws.
 *
 * se_mix_snr: get_noisy_data for B items at once. clean [B, Lc], noise [B, Ln]
 * (one clip per item). Device int arrays from the host RNG: noise_start[B]
 * (crop start when Ln > Lc, :88-93), snr_db[B] (randint(-20, 20), :98),
 * nplace[B] (< 0: tiled repeat over floor(Lc/Ln')*Ln' samples, noise_repeat
 * None, :116-121; >= 0: that many placements place[b*R + r] added in order,
 * :108-115). scale[B] = (clean_rms / 10^(snr/20)) / noise_rms (:95-100);
 * repeat_noise [B, Lc]; mix = clean + repeat_noise [B, Lc] (:123).
 * se_crop_pad: AudioSpliter.split + default_collate over a ragged batch:
 * out[b, t] = src[off[b] + start[b] + t] if start[b] + t < len[b] else 0,
 * t < chunk (pad when len < chunk with start 0; crop at the host's random
 * start otherwise). off, len, start: device arrays.
 * se_pcm16_to_float: x / 32768 (torchaudio.load's normalisation);
 * se_float_to_pcm16: clamp(rint(x * 32768), -32768, 32767) (PCM_S 16 save).
 * ------------------------------------------------------------------------ */
int se_mix_snr(const float* clean, const float* noise, int B, int Lc, int Ln,
               const int* noise_start, const int* snr_db, const int* place,
               const int* nplace, int R, float* mix, float* repeat_noise,
               float* scale, void* stream);
int se_crop_pad(const float* src, const long long* off, const int* len,
                const int* start, int B, int chunk, float* out, void* stream);
int se_pcm16_to_float(const int16_t* in, long long n, float* out, void* stream);
int se_float_to_pcm16(const float* in, long long n, int16_t* out, void* stream);

/* se_resample: mix_audio.py:71-77 (torchaudio.transforms.Resample(orig, new),
 * default sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99) as a
 * polyphase FIR: x [rows, L] -> out [rows, Lout], Lout = ceil(new * L / orig);
 * orig / nw are the rates divided by their gcd; kern [nw][K] (K = 2 width + orig)
 * is the windowed-sinc table built by the host (sehip.data.resample_kernel). */
int se_resample(const float* x, int rows, int L, int orig, int nw, const float* kern, int K, int width,
                float* out, int Lout, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SEHIP_H */
