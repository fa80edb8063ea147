"""The models' glue as HIP passes (csrc/glue.hip, ABI 10), each a differentiable op.

The reference's forwards are written with torch layout and elementwise calls
between the convs (.contiguous() of a permuted view, .float() / .to(dtype),
torch.cat / chunk / stack, sigmoid * x, clamp_); on the product path those are
these ops instead, so a step launches no ATen kernel:

* contiguous(x, dtype): a strided copy with the storage-type conversion fused
  (se_copy_strided); its backward is the cast back.
* stack(tensors, dtype): torch.stack([t.to(dtype) ...]) as one copy per tensor.
* clamp(x, lo, hi): torch.clamp_(x, lo, hi) of the models' waveform output.
* complex_lstm_combine / _stack_re_im: ComplexLSTM's re / im bookkeeping
  (complex_nn.py:128-142) around the stacked recurrence.
* carn_mask, add_sigmoid, gate_cat, glu: CARN / GCARN (carn.py:9-27, 59-76,
  107-113, 161-168).
* chunk_split / chunk_overlap_add: sehip/longform.py's chunking (config 5).
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N

_LL5 = ctypes.c_longlong * 5


def copy_into(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst[...] = src[...] (same shape, any strides, storage types converted) in one launch."""
    if tuple(src.shape) != tuple(dst.shape):
        raise ValueError(f"sehip copy: shapes {tuple(src.shape)} and {tuple(dst.shape)} differ")
    N.require_device(src, dtype=src.dtype)
    N.require_device(dst, dtype=dst.dtype)
    shape, ss, ds = list(src.shape), list(src.stride()), list(dst.stride())
    # drop unit dims, then merge dims that are contiguous in both tensors
    dims = [(n, a, b) for n, a, b in zip(shape, ss, ds) if n != 1] or [(1, 0, 0)]
    merged = [dims[0]]
    for n, a, b in dims[1:]:
        pn, pa, pb = merged[-1]
        if pa == a * n and pb == b * n:
            merged[-1] = (pn * n, a, b)
        else:
            merged.append((n, a, b))
    if len(merged) > 5:
        raise RuntimeError("sehip copy: more than 5 non-mergeable dims")
    nd = len(merged)
    N.check(N.lib().se_copy_strided(src.data_ptr(), N.dtype_code(src), dst.data_ptr(), N.dtype_code(dst), nd,
                                    _LL5(*[m[0] for m in merged]), _LL5(*[m[1] for m in merged]),
                                    _LL5(*[m[2] for m in merged]), N.stream_of(dst)), "se_copy_strided")
    return dst


class _Contig(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src_dtype = x.dtype
        return copy_into(x, torch.empty(x.shape, device=x.device, dtype=dtype))

    @staticmethod
    def backward(ctx, g):
        if g.dtype == ctx.src_dtype:
            return g, None
        return copy_into(g, torch.empty(g.shape, device=g.device, dtype=ctx.src_dtype)), None


def contiguous(x: torch.Tensor, dtype=None) -> torch.Tensor:
    """x.contiguous().to(dtype) as one HIP pass (x itself when nothing changes)."""
    dtype = dtype or x.dtype
    if x.is_contiguous() and x.dtype == dtype:
        return x
    return _Contig.apply(x, dtype)


class _Stack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dtype, *ts):
        out = torch.empty((len(ts),) + tuple(ts[0].shape), device=ts[0].device, dtype=dtype)
        for i, t in enumerate(ts):
            copy_into(t, out[i])
        ctx.dtypes = [t.dtype for t in ts]
        return out

    @staticmethod
    def backward(ctx, g):
        outs = []
        for i, dt in enumerate(ctx.dtypes):
            gi = g[i]   # a view of the stacked gradient: disjoint storage per tensor
            outs.append(gi if dt == g.dtype else copy_into(gi, torch.empty(gi.shape, device=g.device, dtype=dt)))
        return (None, *outs)


def stack(ts, dtype=None) -> torch.Tensor:
    """torch.stack([t.to(dtype) for t in ts]) (HIP copies; each gradient a view of the stacked one)."""
    return _Stack.apply(dtype or ts[0].dtype, *ts)


class _Clamp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lo, hi):
        N.require_device(x, dtype=x.dtype)
        x = x.contiguous()
        y = torch.empty_like(x)
        N.check(N.lib().se_clamp_fwd(x.data_ptr(), y.data_ptr(), x.numel(), float(lo), float(hi), N.dtype_code(x),
                                     N.stream_of(x)), "se_clamp_fwd")
        ctx.save_for_backward(x)
        ctx.lim = (float(lo), float(hi))
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = g.contiguous()
        dx = torch.empty_like(x)
        N.check(N.lib().se_clamp_bwd(g.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), *ctx.lim,
                                     N.dtype_code(x), N.stream_of(g)), "se_clamp_bwd")
        return dx, None, None


def clamp(x, lo, hi):
    """torch.clamp_(x, lo, hi) of a model's output waveform (frcrn.py:154, dccrn.py:211, carn.py:170,
    dcunet.py:188): the values and gradient of the reference's in-place clamp (gradient where
    lo <= x <= hi), as one HIP pass each way."""
    return _Clamp.apply(x, lo, hi)


# --------------------------------------------------------------------------- ComplexLSTM
class _StackReIm(torch.autograd.Function):
    """x [B, T, 2I] (any dense layout, any storage type) -> fp32 [2B, T, I]: the real
    half's sequences then the imaginary half's (complex_nn.py:128-131 + the batch stack).
    The input gradient is written in x's own layout (e.g. the transposed view of a conv
    output), so the producer's backward receives it contiguous."""

    @staticmethod
    def forward(ctx, x):
        B, T, I2 = x.shape
        I = I2 // 2
        out = torch.empty((2, B, T, I), device=x.device, dtype=torch.float32)
        sb, st, sk = x.stride()
        src = torch.as_strided(x, (2, B, T, I), (I * sk, sb, st, sk))
        copy_into(src, out)
        dense = x.is_contiguous() or x.transpose(1, 2).is_contiguous()
        ctx.shape, ctx.dtype = (B, T, I2), x.dtype
        ctx.strides = x.stride() if dense else (T * I2, I2, 1)
        return out.view(2 * B, T, I)

    @staticmethod
    def backward(ctx, g):
        B, T, I2 = ctx.shape
        I = I2 // 2
        sb, st, sk = ctx.strides
        dx = torch.empty_strided((B, T, I2), ctx.strides, device=g.device, dtype=ctx.dtype)
        dst = torch.as_strided(dx, (2, B, T, I), (I * sk, sb, st, sk))
        copy_into(g.reshape(2, B, T, I), dst)
        return dx


def stack_re_im(x):
    return _StackReIm.apply(x)


class _CLstmCombine(torch.autograd.Function):
    """h [2, 2B, T, H] fp32 (real_lstm, imag_lstm over [re; im]) -> [B, T, 2H] in `dtype`:
    (real(re) - imag(im), imag(re) + real(im)) (complex_nn.py:134-142). feature_major: the
    result is the transposed view of a [B, 2H, T] storage (the conv layout the caller
    transposes it back to)."""

    @staticmethod
    def forward(ctx, h, dtype, feature_major):
        _, B2, T, H = h.shape
        B = B2 // 2
        h = h.contiguous()
        if feature_major:
            out = torch.empty((B, 2 * H, T), device=h.device, dtype=dtype).transpose(1, 2)
        else:
            out = torch.empty((B, T, 2 * H), device=h.device, dtype=dtype)
        N.check(N.lib().se_complex_lstm_combine_fwd(h.data_ptr(), h.stride(0), B, T, H, out.data_ptr(),
                                                    *out.stride(), N.dtype_code(out), N.stream_of(h)),
                "se_complex_lstm_combine_fwd")
        ctx.geom = (B, T, H)
        return out

    @staticmethod
    def backward(ctx, g):
        B, T, H = ctx.geom
        if g.stride(2) != 1 and g.stride(1) != 1:
            g = contiguous(g)
        dh = torch.empty((2, 2 * B, T, H), device=g.device, dtype=torch.float32)
        N.check(N.lib().se_complex_lstm_combine_bwd(g.data_ptr(), *g.stride(), B, T, H, N.dtype_code(g),
                                                    dh.data_ptr(), dh.stride(0), N.stream_of(g)),
                "se_complex_lstm_combine_bwd")
        return dh, None, None


def complex_lstm_combine(h, dtype, feature_major=False):
    return _CLstmCombine.apply(h, dtype, bool(feature_major))


# --------------------------------------------------------------------------- CARN
class _CarnMask(torch.autograd.Function):
    @staticmethod
    def forward(ctx, m, spec, half):
        B, T = m.shape[0], m.shape[-1]
        m = m.contiguous()
        spec = spec.contiguous()
        est = torch.empty((B, 2 * half, T), device=m.device, dtype=m.dtype)
        N.check(N.lib().se_carn_mask_fwd(m.data_ptr(), m.stride(0), spec.data_ptr(), B, half, T, N.dtype_code(m),
                                         est.data_ptr(), N.stream_of(m)), "se_carn_mask_fwd")
        ctx.save_for_backward(m, spec)
        ctx.half = half
        return est

    @staticmethod
    def backward(ctx, g):
        m, spec = ctx.saved_tensors
        g = g.contiguous()
        B, T = m.shape[0], m.shape[-1]
        dm = torch.empty((B, 2, ctx.half, T), device=g.device, dtype=g.dtype)
        dspec = torch.empty_like(spec) if ctx.needs_input_grad[1] else None
        N.check(N.lib().se_carn_mask_bwd(g.data_ptr(), m.data_ptr(), m.stride(0), spec.data_ptr(), B, ctx.half, T,
                                         N.dtype_code(g), dm.data_ptr(), N.ptr(dspec), N.stream_of(g)),
                "se_carn_mask_bwd")
        return dm.view(m.shape), dspec, None


def carn_mask(m, spec, half):
    """CARN's mask + concat (carn.py:161-168): m [B, 2, half, T] (mask re / im), spec the
    ConvSTFT output [B, 2 half, T] -> est [B, 2 half, T], one HIP pass each way."""
    N.require_device(m, spec, dtype=m.dtype)
    return _CarnMask.apply(m, spec, int(half))


class _AddSigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.check(N.lib().se_add_sigmoid_fwd(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), N.dtype_code(a),
                                           N.stream_of(a)), "se_add_sigmoid_fwd")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        g = g.contiguous()
        dz = torch.empty_like(y)
        N.check(N.lib().se_sigmoid_bwd(g.data_ptr(), y.data_ptr(), dz.data_ptr(), y.numel(), N.dtype_code(y),
                                       N.stream_of(g)), "se_sigmoid_bwd")
        return dz, dz


def add_sigmoid(a, b):
    """torch.sigmoid(a + b) (carn.py:70-72) in one pass each way."""
    N.require_device(a, b, dtype=a.dtype)
    if a.shape != b.shape:
        raise ValueError("sehip add_sigmoid: shapes differ")
    return _AddSigmoid.apply(a, b)


class _GateCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, c, skip):
        c, skip = c.contiguous(), skip.contiguous()
        B, C = skip.shape[0], skip.shape[1]
        HW = skip[0, 0].numel()
        out = torch.empty((B, 2 * C) + tuple(skip.shape[2:]), device=skip.device, dtype=skip.dtype)
        N.check(N.lib().se_gate_cat_fwd(c.data_ptr(), skip.data_ptr(), out.data_ptr(), B, C, HW,
                                        N.dtype_code(skip), N.stream_of(skip)), "se_gate_cat_fwd")
        ctx.save_for_backward(c, skip)
        return out

    @staticmethod
    def backward(ctx, g):
        c, skip = ctx.saved_tensors
        g = g.contiguous()
        B, C = skip.shape[0], skip.shape[1]
        dc, dskip = torch.empty_like(c), torch.empty_like(skip)
        N.check(N.lib().se_gate_cat_bwd(g.data_ptr(), c.data_ptr(), skip.data_ptr(), dc.data_ptr(), dskip.data_ptr(),
                                        B, C, skip[0, 0].numel(), N.dtype_code(skip), N.stream_of(g)),
                "se_gate_cat_bwd")
        return dc, dskip


def gate_cat(c, skip):
    """torch.cat([torch.sigmoid(c) * skip, skip], dim=1) (carn.py:74-76 + 112-113), one pass each way."""
    N.require_device(c, skip, dtype=skip.dtype)
    if c.shape != skip.shape:
        raise ValueError("sehip gate_cat: shapes differ")
    return _GateCat.apply(c, skip)


class _Glu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.check(N.lib().se_glu_fwd(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), N.dtype_code(a),
                                   N.stream_of(a)), "se_glu_fwd")
        ctx.save_for_backward(a, b)
        return y

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da, db = torch.empty_like(a), torch.empty_like(b)
        N.check(N.lib().se_glu_bwd(g.data_ptr(), a.data_ptr(), b.data_ptr(), da.data_ptr(), db.data_ptr(), a.numel(),
                                   N.dtype_code(a), N.stream_of(g)), "se_glu_bwd")
        return da, db


def glu(a, b):
    """a * torch.sigmoid(b) (ConvGLU / DeConvGLU, carn.py:9-27), one pass each way."""
    N.require_device(a, b, dtype=a.dtype)
    if a.shape != b.shape:
        raise ValueError("sehip glu: shapes differ")
    return _Glu.apply(a, b)


# --------------------------------------------------------------------------- long-form chunks
def chunk_split(wav: torch.Tensor, chunk: int, starts) -> torch.Tensor:
    """[L] -> [n, chunk] chunks at the given (uniformly spaced) starts, zero past the end."""
    x = wav.reshape(-1).contiguous()
    N.require_device(x, dtype=x.dtype)
    n = len(starts)
    hop = starts[1] - starts[0] if n > 1 else chunk
    out = torch.empty((n, chunk), device=x.device, dtype=x.dtype)
    N.check(N.lib().se_chunk_split(x.data_ptr(), x.numel(), n, chunk, hop, N.dtype_code(x), out.data_ptr(),
                                   N.stream_of(x)), "se_chunk_split")
    return out


def chunk_overlap_add(y: torch.Tensor, chunk: int, overlap: int, length: int) -> torch.Tensor:
    """[n, width] enhanced chunks -> [length] with sehip/longform.py's linear cross-fade."""
    y = y.contiguous()
    N.require_device(y, dtype=y.dtype)
    n, width = y.shape
    out = torch.empty(length, device=y.device, dtype=y.dtype)
    N.check(N.lib().se_chunk_overlap_add(y.data_ptr(), n, width, chunk, overlap, length, N.dtype_code(y),
                                         out.data_ptr(), N.stream_of(y)), "se_chunk_overlap_add")
    return out
