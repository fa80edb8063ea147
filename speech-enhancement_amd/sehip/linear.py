"""nn.Linear / ComplexLinear on the hand-written GEMM (se_gemm, csrc/gemm.hip).

Replaces the two nn.Linear calls of ComplexLinear (complex_nn.py:93-113, DCCRN's
LSTMBlock dccrn.py:71-86) and CARN's Linear(512 -> 514) head (carn.py:133,
157-159): forward, input gradient, weight gradient and bias gradient, for fp32
(split-fp16 MFMA, fp32-class) and bf16 / fp16 storage (the one-term MFMA of that
format, nn.Linear's own arithmetic: exact products, fp32 accumulation, one
rounding). The nn.Linear modules stay the parameter holders (state_dict keys
unchanged); only their forward is never called.

Layouts. The input is a 3-D [Bx, Tx, in] view whose features are either the
contiguous axis ("rows": x[b, t, :] contiguous) or whose time axis is
("features": x[b, :, t] at stride 1, e.g. h.reshape(b, c*f, t).transpose(1, 2),
the models' hand-off from a conv stack to a Linear). The GEMMs read both forms
in place, so the reference's permute / transpose copies around the Linear
disappear. The output is produced in either form too (``feature_major_out``):
a [Bx, out, Tx] storage returned as its transposed [Bx, Tx, out] view, which is
the layout the consumer (a conv over [B, C, F, T]) reads without a copy.
With ``halves`` = 2 the input's last axis is split in two equal halves, each
mapped by its own weight (real_linear on the first, imag_linear on the second),
the two outputs concatenated on the last axis: ComplexLinear's "no cross terms"
form (complex_nn.py:106-113) in place, without the chunk / cat.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import functional as F
from . import glue


def _layout3(x: torch.Tensor):
    """(x3, strides (sb, st, sk)) of x viewed as a dense [Bx, Tx, K]: contiguous ("rows") or the
    transposed view of a contiguous [Bx, K, Tx] ("features"); None for any other layout (the
    GEMMs' scale pass reads the tensor as its numel() contiguous elements)."""
    if x.dim() == 3:
        if x.is_contiguous() or x.transpose(1, 2).is_contiguous():
            return x, x.stride()
        return None
    if x.dim() >= 1 and x.is_contiguous():
        x3 = x.view(1, -1, x.shape[-1])
        return x3, x3.stride()
    return None


def _gemm_calls_fwd(x3, xs, w, b, y3, ys, h, cin, cout, amax):
    Bx, Tx, _ = x3.shape
    sxb, sxt, sxk = xs
    syb, syt, syn = ys
    xa, wa = amax
    if syn == 1:   # rows out: C(m = t, n)
        merge = Bx > 1 and sxb == Tx * sxt and syb == Tx * syt and sxk == 1
        M, bt = (Bx * Tx, 1) if merge else (Tx, Bx)
        F.gemm(x3, w, y3, M=M, N=cout, K=cin, lda=sxt if sxk == 1 else sxk, ldb=cin, ldc=syt,
               a_mcontig=sxk != 1, batches=bt, stride_a=sxb, stride_c=syb, bias0=b, amax_a=xa, amax_b=wa,
               offsets=(h * cin * sxk, 0, h * cout))
    else:          # features out: C(m = n, n' = t)
        F.gemm(w, x3, y3, M=cout, N=Tx, K=cin, lda=cin, ldb=sxt if sxk == 1 else sxk, ldc=syn,
               b_ncontig=sxk != 1, batches=Bx, stride_b=sxb, stride_c=syb, bias0=b, bias_rows=True,
               amax_a=wa, amax_b=xa, offsets=(0, h * cin * sxk, h * cout * syn))


class _LinearHalves(torch.autograd.Function):
    """y = cat_h(x_h W_h^T + b_h) over `halves` equal splits of x's last axis (see module doc)."""

    @staticmethod
    def forward(ctx, x, feature_major_out, halves, *wb):
        ws, bs = wb[0::2], wb[1::2]
        lay = _layout3(x)
        if lay is None:
            x = glue.contiguous(x)
            lay = _layout3(x)
        x3, xs = lay
        cout, cin = ws[0].shape
        Bx, Tx, K = x3.shape
        feature_major_out = feature_major_out and x.dim() == 3
        if K != halves * cin:
            raise RuntimeError(f"sehip linear: input features {K}, weights expect {halves} x {cin}")
        N.require_device(x3, *ws, *bs, dtype=x3.dtype)
        dev, dt = x3.device, x3.dtype
        f32 = dt == torch.float32
        if feature_major_out:
            y = torch.empty((Bx, halves * cout, Tx), device=dev, dtype=dt)
            y3 = y.transpose(1, 2)
        else:
            y3 = torch.empty((Bx, Tx, halves * cout), device=dev, dtype=dt)
        xa = F.amax_of(x3) if f32 else None
        was = [F.amax_of(w) if f32 else None for w in ws]
        for h in range(halves):
            _gemm_calls_fwd(x3, xs, ws[h], bs[h], y3, y3.stride(), h, cin, cout, (xa, was[h]))
        ctx.save_for_backward(x3, *ws)
        ctx.cfg = (halves, [b is not None for b in bs], tuple(x.shape))
        ctx.amax = (xa, was)
        return y3.view(x.shape[:-1] + (halves * cout,)) if x.dim() != 3 else y3

    @staticmethod
    def backward(ctx, gy):
        x3, *ws = ctx.saved_tensors
        halves, has_b, xshape = ctx.cfg
        xa, was = ctx.amax
        cout, cin = ws[0].shape
        Bx, Tx, _ = x3.shape
        sxb, sxt, sxk = x3.stride()
        g3 = gy.reshape(Bx, Tx, halves * cout) if gy.dim() != 3 else gy
        gl = _layout3(g3)
        if gl is None or g3.dtype != x3.dtype:
            g3 = glue.contiguous(g3, x3.dtype)
            gl = _layout3(g3)
        g3, (sgb, sgt, sgn) = gl
        f32 = x3.dtype == torch.float32
        ga = F.amax_of(g3) if f32 else None
        dx = None
        grads = []
        if ctx.needs_input_grad[0]:
            if sxk == 1:
                dx = torch.empty((Bx, Tx, halves * cin), device=x3.device, dtype=x3.dtype)
            else:
                dx = torch.empty((Bx, halves * cin, Tx), device=x3.device, dtype=x3.dtype).transpose(1, 2)
            sdb, sdt, sdk = dx.stride()
            for h in range(halves):
                if sdk == 1:   # dx rows: C(m = t, n' = k), A = g (m = t, kk = n)
                    merge = Bx > 1 and sgb == Tx * sgt and sdb == Tx * sdt and sgn == 1
                    M, bt = (Bx * Tx, 1) if merge else (Tx, Bx)
                    F.gemm(g3, ws[h], dx, M=M, N=cin, K=cout, lda=sgt if sgn == 1 else sgn, ldb=cin, ldc=sdt,
                           a_mcontig=sgn != 1, b_ncontig=True, batches=bt, stride_a=sgb, stride_c=sdb,
                           amax_a=ga, amax_b=was[h], offsets=(h * cout * sgn, 0, h * cin))
                else:          # dx features: C(m = k, n' = t), A = W^T, B = g (kk = n, n' = t)
                    F.gemm(ws[h], g3, dx, M=cin, N=Tx, K=cout, lda=cin, ldb=sgn if sgt == 1 else sgt, ldc=sdk,
                           a_mcontig=True, b_ncontig=sgt == 1, batches=Bx, stride_b=sgb, stride_c=sdb,
                           amax_a=was[h], amax_b=ga, offsets=(0, h * cout * sgn, h * cin * sdk))
            dx = dx.reshape(xshape) if len(xshape) != 3 else dx
        for h in range(halves):
            dw = db = None
            if ctx.needs_input_grad[3 + 2 * h]:
                dw = torch.empty_like(ws[h])
                merge = Bx > 1 and sgb == Tx * sgt and sxb == Tx * sxt
                K, bt = (Bx * Tx, 1) if merge else (Tx, Bx)
                # C(m = n, n' = k) = sum_t g(t, n) x(t, k)
                F.gemm(g3, x3, dw, M=cout, N=cin, K=K, lda=sgn if sgt == 1 else sgt, ldb=sxk if sxt == 1 else sxt,
                       ldc=cin, a_mcontig=sgt != 1, b_ncontig=sxt != 1, batches=bt, sum_batches=bt > 1,
                       stride_a=sgb, stride_b=sxb, amax_a=ga, amax_b=xa,
                       offsets=(h * cout * sgn, h * cin * sxk, 0))
            if has_b[h] and ctx.needs_input_grad[4 + 2 * h]:
                db = torch.empty(cout, device=g3.device, dtype=g3.dtype)
                lib = N.lib()
                wsz = F._workspace(lib.se_bias_grad_workspace_size(Bx, Tx, cout), g3.device)
                N.check(lib.se_bias_grad(g3.data_ptr() + g3.element_size() * h * cout * sgn, Bx, Tx, cout, sgb, sgt,
                                         sgn, N.dtype_code(g3), db.data_ptr(), wsz.data_ptr(), wsz.numel(),
                                         N.stream_of(g3)), "se_bias_grad")
            grads += [dw, db]
        return (dx, None, None, *grads)


LINEAR_CALLS = [0]   # Linear layers run on se_gemm (diagnostics / tests)


def linear_halves(x, weights, biases, feature_major_out=False):
    """cat_h(x_h @ W_h^T + b_h) on se_gemm for a CUDA x of the weights' dtype; x_h the h-th of
    len(weights) equal splits of x's last axis."""
    wb = []
    for w, b in zip(weights, biases):
        wb += [w, b]
    LINEAR_CALLS[0] += 1
    return _LinearHalves.apply(x, bool(feature_major_out), len(weights), *wb)


def linear(x, module: torch.nn.Linear, feature_major_out=False):
    """module(x) (nn.Linear) on se_gemm."""
    return linear_halves(x, [module.weight], [module.bias], feature_major_out)
