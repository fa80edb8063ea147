"""Autograd functions over the sehip C ABI (include/sehip.h).

Each Function validates shapes on the host, allocates outputs and workspace
through PyTorch's caching allocator, and launches on the caller's current
HIP stream. There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import contextlib
import os

import torch
from torch.multiprocessing.reductions import StorageWeakRef

from . import _native as N
_NAT = N


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# Deferred weight-grads: inside deferred_weight_grads(), every conv weight-grad
# GEMM runs on a side HIP stream, so the (LDS/MFMA-bound) weight-grad of layer i
# overlaps the data-grad chain and the HBM-bound CBN / CCBAM backward kernels of
# the following layers on the main stream. Leaving the context makes the
# current stream wait for the side stream (before clip_grad_norm / the
# optimizer read the gradients).
_DEFER: set | None = None
_DEFER_STREAMS: dict = {}
# every side stream the path launches on (deferred weight-grads, CCBAM gates): the
# OpTimer marks calls on them, whose event spans share the CUs with the main stream
SIDE_STREAMS: list = []
# set by sehip.train.wrap_ddp when a hook-based torch DDP wraps the model: its
# per-parameter gradient hooks rule out the side streams (frcrn._overlap_ok)
DDP_HOOKS: list = [False]


@contextlib.contextmanager
def deferred_weight_grads(enabled: bool = True):
    """Use around loss.backward() when every parameter .grad is None on entry
    (zero_grad(set_to_none=True)) and no hook reads gradients during backward
    (not under DDP): autograd sees the weight gradients as produced on the
    current stream, and nothing may read them before the context exits."""
    global _DEFER
    if not enabled or _DEFER is not None:
        yield
        return
    _DEFER = set()
    try:
        yield
    finally:
        pending, _DEFER = _DEFER, None
        for side in pending:
            torch.cuda.current_stream(side.device).wait_stream(side)


def _wgrad_stream(*inputs):
    """Context for a weight-grad launch: a no-op, or (deferred_weight_grads) the
    device's side stream, after it waited for the current stream; the inputs are
    recorded as used on it so the allocator keeps them until it is done."""
    if _DEFER is None:
        return contextlib.nullcontext()
    dev = inputs[0].device
    side = _DEFER_STREAMS.get(dev)
    if side is None:
        side = _DEFER_STREAMS[dev] = torch.cuda.Stream(dev)
        SIDE_STREAMS.append(side)
    side.wait_stream(torch.cuda.current_stream(dev))
    for t in inputs:
        if t is not None:
            t.record_stream(side)
    _DEFER.add(side)
    return torch.cuda.stream(side)


class OpTimer:
    """Live per-entry-point timing with HIP events on the launching stream
    (used by bench.py for the roofline numbers). Disabled unless installed
    with set_op_timer(); then every C-ABI call in this module is bracketed by
    two events and tagged with its algorithmic FLOPs and bytes."""

    def __init__(self):
        self.records = []   # (tag, start_event, end_event, flops, bytes)

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, tag, start, flops=0.0, nbytes=0.0):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        cur = torch.cuda.current_stream()
        side = any(cur == t for t in SIDE_STREAMS)
        self.records.append((tag, start, ev, float(flops), float(nbytes), side))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for tag, a, b, fl, nb, side in self.records:
            d = out.setdefault(tag, dict(calls=0, ms=0.0, flops=0.0, bytes=0.0, side_calls=0))
            d["calls"] += 1
            d["side_calls"] += int(side)   # on a side stream, sharing the CUs with the main one
            d["ms"] += a.elapsed_time(b)
            d["flops"] += fl
            d["bytes"] += nb
        return out


_TIMER: OpTimer | None = None

# MFMA form of the conv GEMMs (se_conv2d_desc.math), per pass: "f32" = exact
# fp32 products on v_mfma_f32_32x32x2_f32; "bf16x3" = split-bf16 operands
# (hi*hi + hi*lo + lo*hi) on v_mfma_f32_32x32x16_bf16, fp32 accumulate.
# "bf16x6" = three-way split, six terms (fp32-class); "bf16" = operands rounded
# to bf16, one term (the low-precision configs' arithmetic: BASELINE configs
# 2/3, judged against the fp32 oracle with the reference's own bf16 drift).
# "f16x3" = per-tensor power-of-two scaled split-fp16 (hi + lo, three terms on
# v_mfma_f32_32x32x16_f16): 22 significant bits per operand, fp32-class
# (tests/test_gpu_conv_x3.py holds every pass at or below the exact-fp32 MFMA
# path's error against fp64) at the MFMA cost of bf16x3.
# Initial value from SEHIP_CONV_MATH ("f32", "bf16x3", or per pass as
# "fwd=bf16x3,data=f32,weight=bf16x3"); set_conv_math() changes it.
_MATH_CODES = {"f32": 0, "bf16x3": 1, "bf16x6": 2, "bf16": 3, "f16x3": 4, "f16": 5}
# storage dtype -> the one-term MFMA math 16-bit storage runs (se_conv2d_desc.dtype)
_STORAGE_MATH = {torch.bfloat16: 3, torch.float16: 5}
_PASSES = ("fwd", "data", "weight")
_CONV_MATH = {p: 0 for p in _PASSES}


def set_conv_math(mode: str, **passes: str) -> None:
    """set_conv_math("bf16x3") sets every pass; keyword overrides per pass
    (fwd=, data=, weight=). A mode string may also be the per-pass form
    "fwd=bf16x3,data=f32,weight=bf16x3"."""
    spec = {}
    if "=" in mode:
        for item in mode.split(","):
            k, v = item.split("=")
            spec[k.strip()] = v.strip()
    else:
        spec = {p: mode for p in _PASSES}
    spec.update(passes)
    for k, v in spec.items():
        if k not in _PASSES:
            raise ValueError(f"conv pass must be one of {_PASSES} (got {k!r})")
        if v not in _MATH_CODES:
            raise ValueError(f"conv math must be one of {sorted(_MATH_CODES)} (got {v!r})")
    for k, v in spec.items():
        _CONV_MATH[k] = _MATH_CODES[v]


# Default: scaled split-fp16 on every pass. It is fp32-class: against fp64, each
# pass at every FRCRN layer shape lands at 0.63-0.70x the exact-fp32 MFMA
# path's own error (tests/test_gpu_conv_x3.py, test_gpu_cconv.py), at the MFMA
# cost of bf16x3. The faster, coarser forms are opt-in (set_conv_math /
# SEHIP_CONV_MATH): "bf16x3" (~7x the fp32 path's per-conv error), and "bf16"
# (the low-precision configs' arithmetic).
DEFAULT_CONV_MATH = "f16x3"
set_conv_math(os.environ.get("SEHIP_CONV_MATH", DEFAULT_CONV_MATH))


def get_conv_math() -> str:
    """The current mode: one name when every pass agrees, else the per-pass form."""
    names = {v: k for k, v in _MATH_CODES.items()}
    modes = [names[_CONV_MATH[p]] for p in _PASSES]
    if len(set(modes)) == 1:
        return modes[0]
    return ",".join(f"{p}={m}" for p, m in zip(_PASSES, modes))


# --------------------------------------------------------------------------
# Scale sources of the SE_MATH_F16X3 GEMMs: an upper bound of max |t| per
# tensor (device fp32 [1]). Producers that pass over a tensor anyway register
# one (ComplexBN forward: its output; ComplexBN backward: its input gradient,
# which is the producing conv's dy; CCBAM: its output); a conv pass that finds
# none computes it with se_amax (one read). Entries are keyed by the tensor's
# address and hold only a weak reference to its storage: an entry matches a
# tensor only while that storage is alive, with the same shape and version
# counter, so neither reuse of freed memory nor an in-place write can pair a
# tensor with a stale bound, and the table keeps nothing alive.
# --------------------------------------------------------------------------
F16X3 = 4
_AMAX: dict = {}


def amax_put(t: torch.Tensor, amax: torch.Tensor) -> None:
    if len(_AMAX) > 256:
        for k in [k for k, e in _AMAX.items() if e[1].expired()]:
            del _AMAX[k]
    _AMAX[t.data_ptr()] = (amax, StorageWeakRef(t.untyped_storage()), tuple(t.shape), t._version)


def amax_get(t: torch.Tensor):
    e = _AMAX.get(t.data_ptr())
    if e is None or e[1].expired() or e[2] != tuple(t.shape) or e[3] != t._version:
        return None
    return e[0]


def amax_of(t: torch.Tensor) -> torch.Tensor:
    """The registered bound of max |t|, else max |t| computed now (and registered)."""
    a = amax_get(t)
    if a is None:
        a = torch.empty(1, device=t.device, dtype=torch.float32)
        N.check(N.lib().se_amax_init(t.data_ptr(), t.numel(), a.data_ptr(), N.stream_of(t)), "se_amax_init")
        amax_put(t, a)
    return a


def amax_pair(x: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """max(bound of x, bound of s) in a fresh slot: the registered bounds (or one read of each
    tensor) combined by the amax kernels themselves (se_amax_init + se_amax on the two slots)."""
    ax, as_ = amax_of(x), amax_of(s)
    out = new_amax(x.device)
    lib, st = N.lib(), N.stream_of(x)
    N.check(lib.se_amax_init(ax.data_ptr(), 1, out.data_ptr(), st), "se_amax_init")
    N.check(lib.se_amax(as_.data_ptr(), 1, out.data_ptr(), st), "se_amax")
    return out


def new_amax(device) -> torch.Tensor:
    return torch.empty(1, device=device, dtype=torch.float32)


def _weight_amax(d, wr, wi):
    """se_conv2d_desc.w_amax for one conv call: one single-workgroup launch in the
    forward, shared by the forward and data-grad GEMMs (which otherwise reduce the
    weights twice each); None where no split-fp16 gather pass reads it."""
    need = ((_pass_math("fwd", d) == F16X3 and d.out_channels > 64)
            or (_pass_math("data", d) == F16X3 and d.in_channels > 64))
    if not need:
        return None
    a = new_amax(wr.device)
    n = wr.numel()
    N.check(N.lib().se_amax_weights(wr.data_ptr(), n, N.ptr(wi), a.data_ptr(), N.stream_of(wr)),
            "se_amax_weights")
    return a


def _f16_operands(d):
    """(x, dy) -> whether a SE_MATH_F16X3 GEMM of this conv reads that operand's
    scale: the split kernels' shape rules of cconv.hip (gather N > 64, weight-grad
    N > 32 and N % 16 == 0)."""
    fwd = _pass_math("fwd", d) == F16X3 and d.out_channels > 64
    data = _pass_math("data", d) == F16X3 and d.in_channels > 64
    n = d.in_channels if d.transposed else d.out_channels
    wgt = _pass_math("weight", d) == F16X3 and n > 32 and n % 16 == 0
    return fwd or wgt, data or wgt


SE_MATH_F32 = 0


def _pass_math(pass_name, d) -> int:
    fm = getattr(d, "force_math", None)
    if fm is not None:   # 16-bit storage: the one-term MFMA of its format on every pass
        return fm
    m = _CONV_MATH[pass_name]
    # a data-fed conv (exact=True: a model's first conv, whose input is the raw spectrum
    # and carries the batch's whole level spread) runs exact fp32 where the mode is the
    # per-tensor-scaled f16x3 (DESIGN.md §3.2 "Dynamic range")
    if m == F16X3 and getattr(d, "exact", False):
        return SE_MATH_F32
    return m


def _gemm_tag(pass_name, d, joined=False):
    """OpTimer tag of a conv pass by the kernel that runs it (cconv.hip's
    dispatch): conv_{fwd,data,wgrad}[_joined]_{f32,f16x3,bf16x3,...,smalln}.
    The decoder's joined passes (se_conv2d_*_joined) are tagged apart: each
    such call is one launch of one kernel instantiation, so the bench can pair
    their live event times with that instantiation's PMC traffic."""
    names = {v: k for k, v in _MATH_CODES.items()}
    tr = bool(d.transposed)
    j = "_joined" if joined else ""
    if pass_name == "weight":
        n = d.in_channels if tr else d.out_channels          # channels of the direct operand
        kind = "smalln" if n <= 8 else (names[_pass_math("weight", d)] if n > 32 else "f32")
        kind = "f32" if kind == "bf16x6" else kind
        return f"conv_wgrad{j}_{kind}"
    n = d.out_channels if pass_name == "fwd" else d.in_channels
    kind = "smalln" if n <= 16 else (names[_pass_math(pass_name, d)] if n > 64 else "f32")
    return f"conv_{pass_name}{j}_{kind}"


def _with_math(d, pass_name):
    d.math = _pass_math(pass_name, d)
    return N.ctypes.byref(d)


def set_op_timer(t: OpTimer | None):
    global _TIMER
    _TIMER = t


def _conv_flops(d) -> float:
    """Algorithmic FLOPs of one pass (= torch FlopCounterMode's conv formula:
    2 * positions * Cin * Cout * kh * kw over the conv's (input for convT,
    output for conv) grid). The fused complex conv does the work of the
    reference's four real convs of Cin/2 x Cout/2 channels exactly."""
    ho, wo = N.c_int(), N.c_int()
    N.lib().se_conv2d_out_shape(N.ctypes.byref(d), N.ctypes.byref(ho), N.ctypes.byref(wo))
    grid = (d.in_h * d.in_w) if d.transposed else (ho.value * wo.value)
    return 2.0 * d.batch * grid * d.in_channels * d.out_channels * d.kernel_h * d.kernel_w


# --------------------------------------------------------------------------
# Complex / real (transposed) conv2d — se_conv2d_* (cconv.hip)
# --------------------------------------------------------------------------
def conv_desc(x_shape, out_channels, kernel, stride, padding, dilation, output_padding,
              transposed, complex_w, padding_end=None, exact=False) -> N.ConvDesc:
    """padding = (top, left) begin padding; padding_end = (bottom, right), or
    None for symmetric padding (nn.Conv2d)."""
    b, cin, h, w = x_shape
    d = N.ConvDesc()
    d.batch, d.in_channels, d.in_h, d.in_w = b, cin, h, w
    d.out_channels = out_channels
    d.kernel_h, d.kernel_w = kernel
    d.stride_h, d.stride_w = stride
    d.pad_h, d.pad_w = padding
    d.dil_h, d.dil_w = dilation
    d.out_pad_h, d.out_pad_w = output_padding
    d.transposed, d.complex_weights = int(transposed), int(complex_w)
    d.pad_h_end, d.pad_w_end = (-1, -1) if padding_end is None else padding_end
    d.exact = bool(exact)   # host-side only (see _pass_math)
    d.math = _pass_math("fwd", d)
    return d


def _prep_data_weights(d, wr, wi, wa):
    """The data-grad weight image of a conv call (se_conv2d_desc.data_weights), built
    in the forward right after the forward GEMM: (uint8 image tensor, data-pass math),
    or None with SEHIP_DATA_PREP=0 or when a split-fp16 data pass has no shared weight
    bound. In the backward the same small prep launch would wait for CU slots behind
    the side stream's weight-grad GEMMs, stalling the main stream."""
    if os.environ.get("SEHIP_DATA_PREP", "1") == "0":
        return None
    m = _pass_math("data", d)
    if m == F16X3 and d.in_channels > 64 and wa is None:
        return None
    lib, fm = N.lib(), d.math
    d.math = m
    try:
        nb = lib.se_conv2d_data_weights_size(N.ctypes.byref(d))
        img = torch.empty(nb, dtype=torch.uint8, device=wr.device)
        N.check(lib.se_conv2d_prep_data_weights(N.ctypes.byref(d), wr.data_ptr(), N.ptr(wi), img.data_ptr(), nb,
                                                N.stream_of(wr)), "se_conv2d_prep_data_weights")
    finally:
        d.math = fm
    return img, m


DATA_IMG_CALLS = [0]   # data-grad passes that read a forward-built weight image (tests)


def _data_weights_of(ctx, d) -> int | None:
    """ctx's prepared data-grad image pointer if it matches the pass's math now."""
    img = getattr(ctx, "data_img", None)
    if img is None or img[1] != _pass_math("data", d):
        return None
    DATA_IMG_CALLS[0] += 1
    return img[0].data_ptr()


def _check_weights(in_channels, out_channels, kernel, transposed, wr, wi, br, bi):
    """The kernels read the weights at the shape the descriptor implies: refuse a mismatch
    the way nn.Conv2d / nn.ConvTranspose2d do (RuntimeError) instead of reading past them.
    conv: [Cout, Cin, kh, kw]; convT: [Cin, Cout, kh, kw]; complex: each of wr / wi at half
    of both channel counts (complex_nn.py:67-91)."""
    h = 2 if wi is not None else 1
    ci, co = in_channels // h, out_channels // h
    want = (ci, co, *kernel) if transposed else (co, ci, *kernel)
    for w in (wr, wi):
        if w is not None and tuple(w.shape) != want:
            raise RuntimeError(f"sehip conv2d: weight of size {list(w.shape)}, expected {list(want)} for an input "
                               f"with {in_channels} channels ({'transposed, ' if transposed else ''}"
                               f"{out_channels} output channels)")
    for b in (br, bi):
        if b is not None and tuple(b.shape) != (co,):
            raise RuntimeError(f"sehip conv2d: bias of size {list(b.shape)}, expected [{co}]")


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wr, wi, br, bi, geom):
        (out_channels, kernel, stride, padding, dilation, output_padding, transposed, complex_w,
         padding_end, exact, force_math) = geom
        N.require_device(x, wr, wi, br, bi, dtype=x.dtype)
        _check_weights(x.shape[1], out_channels, kernel, transposed, wr, wi, br, bi)
        x = x.contiguous()
        d = conv_desc(tuple(x.shape), out_channels, kernel, stride, padding, dilation,
                      output_padding, transposed, complex_w, padding_end, exact)
        d.force_math = force_math
        d.dtype = N.dtype_code(x)
        d.math = _pass_math("fwd", d)
        lib = N.lib()
        ho, wo = N.c_int(), N.c_int()
        N.check(lib.se_conv2d_out_shape(N.ctypes.byref(d), N.ctypes.byref(ho), N.ctypes.byref(wo)),
                "se_conv2d_out_shape")
        y = torch.empty((x.shape[0], out_channels, ho.value, wo.value), device=x.device, dtype=x.dtype)
        nbytes = lib.se_conv2d_workspace_size(N.ctypes.byref(d))
        ws = _workspace(nbytes, x.device)
        xa = amax_of(x) if _f16_operands(d)[0] else None
        d.x_amax = N.ptr(xa)
        wa = _weight_amax(d, wr, wi)
        d.w_amax = N.ptr(wa)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_conv2d_fwd(_with_math(d, "fwd"), x.data_ptr(), wr.data_ptr(), N.ptr(wi), N.ptr(br),
                                  N.ptr(bi), y.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_of(x)),
                "se_conv2d_fwd")
        if t0 is not None:   # bytes: x read + y written + the weights, once
            _TIMER.end(_gemm_tag("fwd", d), t0, _conv_flops(d),
                       x.element_size() * (x.numel() + y.numel() + wr.numel() * (2 if wi is not None else 1)))
        ctx.save_for_backward(x, wr, wi)
        ctx.desc, ctx.nbytes, ctx.has_bias, ctx.x_amax, ctx.w_amax = d, nbytes, br is not None, xa, wa
        ctx.data_img = _prep_data_weights(d, wr, wi, wa) if ctx.needs_input_grad[0] else None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wr, wi = ctx.saved_tensors
        gy = gy.contiguous()
        d, lib = ctx.desc, N.lib()
        ws = _workspace(ctx.nbytes, gy.device)
        ga = amax_of(gy) if _f16_operands(d)[1] else None
        d.x_amax, d.dy_amax, d.w_amax = N.ptr(ctx.x_amax), N.ptr(ga), N.ptr(ctx.w_amax)
        dx = dwr = dwi = dbr = dbi = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            d.data_weights = _data_weights_of(ctx, d)
            t0 = _TIMER.begin() if _TIMER else None
            N.check(lib.se_conv2d_bwd_data(_with_math(d, "data"), gy.data_ptr(), wr.data_ptr(), N.ptr(wi),
                                           dx.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_of(gy)),
                    "se_conv2d_bwd_data")
            d.data_weights, ctx.data_img = None, None
            if t0 is not None:
                _TIMER.end(_gemm_tag("data", d), t0, _conv_flops(d),
                           4.0 * (gy.numel() + dx.numel() + wr.numel() * (2 if wi is not None else 1)))
        if any(ctx.needs_input_grad[1:5]):
            # a conv without an input gradient (a model's first conv) is the last one in
            # the backward: its weight-grad runs on the current stream, beside the side
            # stream's still-queued weight-grads, instead of behind them
            last = not ctx.needs_input_grad[0]
            with contextlib.nullcontext() if last else _wgrad_stream(x, gy, ctx.x_amax, ga):
                if _DEFER is not None and not last:
                    ws = _workspace(ctx.nbytes, gy.device)
                if ctx.x_amax is None and _f16_operands(d)[0]:   # mode changed since forward
                    d.x_amax = N.ptr(amax_of(x))
                dwr = torch.empty_like(wr)
                dwi = torch.empty_like(wi) if wi is not None else None
                if ctx.has_bias:
                    nb = d.out_channels // 2 if d.complex_weights else d.out_channels
                    dbr = torch.empty(nb, device=gy.device, dtype=gy.dtype)
                    dbi = torch.empty(nb, device=gy.device, dtype=gy.dtype) if d.complex_weights else None
                t0 = _TIMER.begin() if _TIMER else None
                N.check(lib.se_conv2d_bwd_weight(_with_math(d, "weight"), x.data_ptr(), gy.data_ptr(),
                                                 dwr.data_ptr(), N.ptr(dwi), N.ptr(dbr), N.ptr(dbi),
                                                 ws.data_ptr(), ws.numel(), N.stream_of(gy)),
                        "se_conv2d_bwd_weight")
                if t0 is not None:
                    _TIMER.end(_gemm_tag("weight", d), t0, _conv_flops(d),
                               4.0 * (x.numel() + gy.numel() + wr.numel() * (2 if wi is not None else 1)))
        return dx, dwr, dwi, dbr, dbi, None


SE_E_UNSUPPORTED = -3


def _join_raw(x, s, cat=False):
    """complex_concat([align(x), s]) materialised (no autograd): the fallback
    of the joined conv passes when no joined kernel covers the mode/shape.
    cat=True: torch.cat([F.pad(x, to s's grid), s]) (DCUNet, dcunet.py:89-93)."""
    B, Cx, Fx, Tx = x.shape
    _, Cs, F_, T = s.shape
    if cat:
        return torch.cat([torch.nn.functional.pad(x, (0, T - Tx, 0, F_ - Fx)), s], dim=1)
    out = torch.empty((B, Cx + Cs, F_, T), device=x.device, dtype=x.dtype)
    N.check(N.lib().se_complex_join(x.data_ptr(), Cx, Fx, Tx, s.data_ptr(), Cs, F_, T, out.data_ptr(), B,
                                    N.dtype_code(x), N.stream_of(x)), "se_complex_join")
    return out


class _ConvJoined(torch.autograd.Function):
    """Complex (transposed) conv over complex_concat([align(x), s]) — the FRCRN
    decoder's trim / pad / concat + ConvTransposeBlock conv (frcrn.py:93-101) —
    or over torch.cat([pad(x), s]) (cat: DCUNet's decoder, dcunet.py:89-93),
    without writing the joined tensor: the forward GEMM gathers from x and s,
    the data-grad epilogue writes dx and ds directly, the weight-grad reads
    both as its D operand (se_conv2d_*_joined). Modes or shapes without a
    joined kernel (SE_E_UNSUPPORTED) materialise the join for that pass.
    force_math (16-bit storage): the one-term MFMA of the storage format, the
    tensors read and written as they are (se_conv2d_desc.dtype)."""

    @staticmethod
    def forward(ctx, x, s, wr, wi, br, bi, geom):
        out_channels, kernel, stride, padding, dilation, output_padding, transposed, cat, force_math = geom
        N.require_device(x, s, wr, wi, br, bi, dtype=x.dtype)
        _check_weights(2 * s.shape[1], out_channels, kernel, transposed, wr, wi, br, bi)
        x, s = x.contiguous(), s.contiguous()
        B, Cs, F_, T = s.shape
        Fx, Tx = x.shape[2], x.shape[3]
        d = conv_desc((B, 2 * Cs, F_, T), out_channels, kernel, stride, padding, dilation,
                      output_padding, transposed, True)
        d.join_cat, d.force_math, d.dtype = int(cat), force_math, N.dtype_code(x)
        d.math = _pass_math("fwd", d)
        es = x.element_size()
        lib = N.lib()
        ho, wo = N.c_int(), N.c_int()
        N.check(lib.se_conv2d_out_shape(N.ctypes.byref(d), N.ctypes.byref(ho), N.ctypes.byref(wo)),
                "se_conv2d_out_shape")
        y = torch.empty((B, out_channels, ho.value, wo.value), device=x.device, dtype=x.dtype)
        nbytes = lib.se_conv2d_workspace_size(N.ctypes.byref(d))
        ws = _workspace(nbytes, x.device)
        st = N.stream_of(x)
        # scale source of the joined input: max of the two sources' bounds
        xa = amax_pair(x, s) if _f16_operands(d)[0] else None
        d.x_amax = N.ptr(xa)
        wa = _weight_amax(d, wr, wi)
        d.w_amax = N.ptr(wa)
        t0 = _TIMER.begin() if _TIMER else None
        rc = lib.se_conv2d_fwd_joined(_with_math(d, "fwd"), x.data_ptr(), Fx, Tx, s.data_ptr(), wr.data_ptr(),
                                      wi.data_ptr(), N.ptr(br), N.ptr(bi), y.data_ptr(), ws.data_ptr(), ws.numel(), st)
        if rc == SE_E_UNSUPPORTED:
            rc = lib.se_conv2d_fwd(N.ctypes.byref(d), _join_raw(x, s, cat).data_ptr(), wr.data_ptr(), wi.data_ptr(),
                                   N.ptr(br), N.ptr(bi), y.data_ptr(), ws.data_ptr(), ws.numel(), st)
        N.check(rc, "se_conv2d_fwd_joined")
        if t0 is not None:
            _TIMER.end(_gemm_tag("fwd", d, joined=True), t0, _conv_flops(d),
                       es * (x.numel() + s.numel() + y.numel() + 2 * wr.numel()))
        ctx.save_for_backward(x, s, wr, wi)
        ctx.desc, ctx.nbytes, ctx.has_bias, ctx.x_amax, ctx.w_amax = d, nbytes, br is not None, xa, wa
        ctx.data_img = (_prep_data_weights(d, wr, wi, wa) if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
                        else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, s, wr, wi = ctx.saved_tensors
        gy = gy.contiguous()
        d, lib = ctx.desc, N.lib()
        Fx, Tx = x.shape[2], x.shape[3]
        ws = _workspace(ctx.nbytes, gy.device)
        st = N.stream_of(gy)
        ga = amax_of(gy) if _f16_operands(d)[1] else None
        xa = ctx.x_amax
        if xa is None and _f16_operands(d)[0]:   # mode changed since forward
            xa = amax_pair(x, s)
        d.x_amax, d.dy_amax, d.w_amax = N.ptr(xa), N.ptr(ga), N.ptr(ctx.w_amax)
        gx = gs = dwr = dwi = dbr = dbi = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gx, gs = torch.empty_like(x), torch.empty_like(s)
            d.data_weights = _data_weights_of(ctx, d)
            t0 = _TIMER.begin() if _TIMER else None
            rc = lib.se_conv2d_bwd_data_joined(_with_math(d, "data"), gy.data_ptr(), wr.data_ptr(), wi.data_ptr(),
                                               gx.data_ptr(), Fx, Tx, gs.data_ptr(), ws.data_ptr(), ws.numel(), st)
            if rc == SE_E_UNSUPPORTED:
                dj = torch.empty((d.batch, d.in_channels, d.in_h, d.in_w), device=gy.device, dtype=gy.dtype)
                N.check(lib.se_conv2d_bwd_data(N.ctypes.byref(d), gy.data_ptr(), wr.data_ptr(), wi.data_ptr(),
                                               dj.data_ptr(), ws.data_ptr(), ws.numel(), st), "se_conv2d_bwd_data")
                if d.join_cat:   # torch.cat order: x's gradient is the first half, cropped to x's grid
                    Cx = x.shape[1]
                    gx.copy_(dj[:, :Cx, :Fx, :Tx])
                    gs.copy_(dj[:, Cx:])
                    rc = 0
                else:
                    rc = lib.se_complex_join_bwd(dj.data_ptr(), gx.data_ptr(), x.shape[1], Fx, Tx, gs.data_ptr(),
                                                 s.shape[1], d.in_h, d.in_w, d.batch, N.dtype_code(gy), st)
            N.check(rc, "se_conv2d_bwd_data_joined")
            d.data_weights, ctx.data_img = None, None
            if t0 is not None:
                _TIMER.end(_gemm_tag("data", d, joined=True), t0, _conv_flops(d),
                           gy.element_size() * (gy.numel() + gx.numel() + gs.numel() + 2 * wr.numel()))
        if any(ctx.needs_input_grad[2:6]):
            with _wgrad_stream(x, s, gy, xa, ga):
                if _DEFER is not None:
                    ws = _workspace(ctx.nbytes, gy.device)
                st = N.stream_of(gy)
                dwr, dwi = torch.empty_like(wr), torch.empty_like(wi)
                if ctx.has_bias:
                    nb = d.out_channels // 2
                    dbr = torch.empty(nb, device=gy.device, dtype=gy.dtype)
                    dbi = torch.empty(nb, device=gy.device, dtype=gy.dtype)
                t0 = _TIMER.begin() if _TIMER else None
                rc = lib.se_conv2d_bwd_weight_joined(_with_math(d, "weight"), x.data_ptr(), Fx, Tx, s.data_ptr(),
                                                     gy.data_ptr(), dwr.data_ptr(), dwi.data_ptr(), N.ptr(dbr),
                                                     N.ptr(dbi), ws.data_ptr(), ws.numel(), st)
                if rc == SE_E_UNSUPPORTED:
                    rc = lib.se_conv2d_bwd_weight(N.ctypes.byref(d), _join_raw(x, s, d.join_cat).data_ptr(), gy.data_ptr(),
                                                  dwr.data_ptr(), dwi.data_ptr(), N.ptr(dbr), N.ptr(dbi),
                                                  ws.data_ptr(), ws.numel(), st)
                N.check(rc, "se_conv2d_bwd_weight_joined")
                if t0 is not None:
                    _TIMER.end(_gemm_tag("weight", d, joined=True), t0, _conv_flops(d),
                               gy.element_size() * (x.numel() + s.numel() + gy.numel() + 2 * wr.numel()))
        return gx, gs, dwr, dwi, dbr, dbi, None


def conv2d_joined(x, s, wr, wi, br=None, bi=None, *, out_channels, kernel, stride=1, padding=0,
                  dilation=1, output_padding=0, transposed=False, cat=False):
    """conv2d(complex_join(x, s), ...) with the join folded into the GEMMs.
    x: [B, C, Fx, Tx] decoder state, s: [B, C, F, T] skip, Fx <= F, Tx >= T
    (frcrn.py:95-99); cat=True: conv2d(torch.cat([F.pad(x, to s's grid), s])) with
    Fx <= F, Tx <= T (DCUNet, dcunet.py:89-93). bf16 / fp16 tensors run natively on the
    one-term MFMA of their format where every pass has a kernel (_native16_ok); other
    storage types run on fp32 copies."""
    if x.shape[1] != s.shape[1] or x.shape[2] > s.shape[2] or (x.shape[3] > s.shape[3] if cat else x.shape[3] < s.shape[3]):
        raise ValueError(f"sehip conv2d_joined: cannot align {tuple(x.shape)} to {tuple(s.shape)}")
    geom = (int(out_channels), _pair(kernel), _pair(stride), _pair(padding), _pair(dilation),
            _pair(output_padding), bool(transposed), bool(cat))
    if x.dtype == torch.float32:
        return _ConvJoined.apply(x, s, wr, wi, br, bi, geom + (None,))
    if x.dtype in _STORAGE_MATH and s.dtype == x.dtype and \
            _native16_ok(x, wr, wi, br, bi, out_channels, transposed, in_channels=2 * s.shape[1]):
        NATIVE16_CALLS[0] += 1
        return _ConvJoined.apply(x, s, wr, wi, br, bi, geom + (_STORAGE_MATH[x.dtype],))
    f32 = lambda t: None if t is None else t.float()
    return _ConvJoined.apply(x.float(), s.float(), f32(wr), f32(wi), f32(br), f32(bi),
                             geom + (_STORAGE_MATH.get(x.dtype),)).to(x.dtype)


NATIVE16_CALLS = [0]   # convs run on 16-bit storage natively (diagnostics / tests)


def _native16_ok(x, wr, wi, br, bi, out_channels, transposed, in_channels=None) -> bool:
    """Whether every pass of a 16-bit-storage conv runs natively (se_conv2d_desc.dtype):
    the weight-grad's direct operand channels N (out for a conv, in for a convT) on the
    one-term split tiles (N % 16 == 0, N > 8) when the weights take a gradient."""
    ts = [t for t in (wr, wi, br, bi) if t is not None]
    if any(t.dtype != x.dtype for t in ts) or os.environ.get("SEHIP_NATIVE16", "1") == "0":
        return False
    if not any(t.requires_grad for t in ts) or not torch.is_grad_enabled():
        return True
    n = (x.shape[1] if in_channels is None else in_channels) if transposed else out_channels
    return n % 16 == 0 and n > 8


def conv2d(x, wr, wi=None, br=None, bi=None, *, out_channels, kernel, stride=1, padding=0,
           dilation=1, output_padding=0, transposed=False, padding_end=None, exact=False):
    """Fused complex conv (wi given) or real conv (wi None) on the HIP path.
    padding is the (top, left) begin padding; padding_end (bottom, right)
    defaults to the same (symmetric, as nn.Conv2d). exact=True: a data-fed conv
    (see _pass_math) whose f16x3 passes run exact fp32 instead.
    bf16 / fp16 tensors (model.to(bfloat16) / .half()) are read and written in their
    own dtype by the one-term MFMA of that format on every pass; shapes those kernels
    do not cover compute the same one-term arithmetic on fp32 copies."""
    base = (int(out_channels), _pair(kernel), _pair(stride), _pair(padding), _pair(dilation),
            _pair(output_padding), bool(transposed), wi is not None,
            None if padding_end is None else _pair(padding_end), bool(exact))
    if x.dtype == torch.float32:
        return _Conv2d.apply(x, wr, wi, br, bi, base + (None,))
    if x.dtype not in _STORAGE_MATH:
        raise RuntimeError(f"sehip conv2d: unsupported storage type {x.dtype}")
    fm = _STORAGE_MATH[x.dtype]
    if _native16_ok(x, wr, wi, br, bi, out_channels, transposed):
        NATIVE16_CALLS[0] += 1
        return _Conv2d.apply(x, wr, wi, br, bi, base + (fm,))
    f32 = lambda t: None if t is None else t.float()
    return _Conv2d.apply(x.float(), f32(wr), f32(wi), f32(br), f32(bi), base + (fm,)).to(x.dtype)


# --------------------------------------------------------------------------
# ComplexBatchNorm2d (+ fused activation) — se_cbn_* (cbn.hip)
# --------------------------------------------------------------------------
ACT_NONE, ACT_LEAKY, ACT_RELU = 0, 1, 2


class _ComplexBN(torch.autograd.Function):
    """ComplexBatchNorm2d (+ fused LeakyReLU / ReLU, or a one-weight nn.PReLU as
    `prelu`) on se_cbn_*. x, the parameters, running statistics and prelu share the
    storage type (fp32, or bf16 / fp16 for model.to(bfloat16) / .half()): the kernels
    read and write that type directly, with fp32 arithmetic and fp64 moments."""

    @staticmethod
    def forward(ctx, x, wrr, wri, wii, br, bi, running, nbt, training, eps, momentum, act, slope,
                fork=False, prelu=None):
        N.require_device(x, dtype=x.dtype)
        N.require_device(wrr, wri, wii, br, bi, prelu, *(running or ()), dtype=x.dtype)
        dt = N.dtype_code(x)
        x = x.contiguous()
        b, c = x.shape[:2]
        hw = x[0, 0].numel()
        y = torch.empty_like(x)
        save = torch.empty(N.CBN_SAVE_FLOATS * (c // 2), device=x.device, dtype=torch.float32)
        params = (wrr, wri, wii, br, bi) if wrr is not None else None
        lib = N.lib()
        ws = _workspace(lib.se_cbn_workspace_size(b, c, hw), x.device)
        mom = -1.0 if momentum is None else float(momentum)
        if prelu is not None:
            act, slope = ACT_LEAKY, 0.0
        # bound of max |y| for an f16x3 consumer (fp32 storage only)
        ya = new_amax(x.device) if training and dt == 0 else None
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_cbn_fwd(x.data_ptr(), y.data_ptr(), b, c, hw,
                               N.ptr_array(params), N.ptr_array(running), N.ptr(nbt),
                               save.data_ptr(), int(training), float(eps), mom, int(act),
                               float(slope), N.ptr(ya), N.ptr(prelu), dt, ws.data_ptr(), ws.numel(),
                               N.stream_of(x)),
                "se_cbn_fwd")
        if ya is not None:
            amax_put(y, ya)
        if t0 is not None:   # 1 read for the moments (training) + 1 read + 1 write
            _TIMER.end("cbn_fwd", t0, 0.0, x.element_size() * x.numel() * (3 if training else 2))
        ctx.save_for_backward(x, save, prelu, *(params or ()))   # y is not needed: se_cbn_bwd recomputes act' from x
        ctx.cfg = (int(training), int(act), float(slope), params is not None)
        if fork:   # (y, alias of y): two consumers, two gradients summed inside se_cbn_bwd2
            ctx.set_materialize_grads(False)
            return y, y.view(y.shape)
        return y

    @staticmethod
    def backward(ctx, gy, gy2=None):
        x, save, prelu, *params = ctx.saved_tensors
        training, act, slope, affine = ctx.cfg
        gate = _ccbam_dx_parts(gy2)   # the CCBAM gate's deferred input gradient (ccbam.py)
        if gate is not None and (gy is None or prelu is not None or x.dtype != torch.float32):
            gy2, gate = ccbam_dx_materialize(gate), None   # no fused form: write it as a tensor
        if gy is None:
            gy, gy2 = gy2, None
        if gy is None:
            return (None,) * 16
        gy = gy.contiguous()
        gy2 = gy2.contiguous() if gy2 is not None and gate is None else None
        dt = N.dtype_code(x)
        b, c = x.shape[:2]
        hw = x[0, 0].numel()
        dx = torch.empty_like(x)
        dparams = [torch.empty_like(p) for p in params] if affine else None
        dprelu = torch.empty_like(prelu) if prelu is not None else None
        lib = N.lib()
        ws = _workspace(lib.se_cbn_workspace_size(b, c, hw), x.device)
        dxa = new_amax(x.device) if training and dt == 0 else None   # bound of max |dx| (the conv's dy)
        t0 = _TIMER.begin() if _TIMER else None
        if gate is not None:
            g, dP, idx, ca, dmean, dmax, amax = gate
            N.check(lib.se_cbn_bwd_ccbam(gy.data_ptr(), g.data_ptr(), dP.data_ptr(), idx.data_ptr(), ca.data_ptr(),
                                         dmean.data_ptr(), dmax.data_ptr(), amax.data_ptr(), x.data_ptr(),
                                         dx.data_ptr(), b, c, hw, N.ptr_array(params if affine else None),
                                         save.data_ptr(), N.ptr_array(dparams), training, act, slope, N.ptr(dxa),
                                         ws.data_ptr(), ws.numel(), N.stream_of(gy)), "se_cbn_bwd_ccbam")
            cur = torch.cuda.current_stream(gy.device)
            for t in gate:   # made on the gate's stream, read here: freed only after this stream's use
                t.record_stream(cur)
            CCBAM_DX_FUSED[0] += 1
        elif gy2 is None:
            N.check(lib.se_cbn_bwd(gy.data_ptr(), None, x.data_ptr(), dx.data_ptr(), b, c, hw,
                                   N.ptr_array(params if affine else None), save.data_ptr(),
                                   N.ptr_array(dparams), training, act, slope, N.ptr(dxa), N.ptr(prelu),
                                   N.ptr(dprelu), dt, ws.data_ptr(), ws.numel(), N.stream_of(gy)), "se_cbn_bwd")
        else:
            N.check(lib.se_cbn_bwd2(gy.data_ptr(), gy2.data_ptr(), x.data_ptr(), dx.data_ptr(), b,
                                    c, hw, N.ptr_array(params if affine else None),
                                    save.data_ptr(), N.ptr_array(dparams), training, act, slope,
                                    N.ptr(dxa), N.ptr(prelu), N.ptr(dprelu), dt, ws.data_ptr(), ws.numel(),
                                    N.stream_of(gy)), "se_cbn_bwd2")
        if dxa is not None:
            amax_put(dx, dxa)
        if t0 is not None:   # (gy [, gy2], x) read twice + dx written
            _TIMER.end("cbn_bwd", t0, 0.0, x.element_size() * x.numel() * (5 if gy2 is None and gate is None else 7))
        g = dparams or [None] * 5
        return (dx, *g, None, None, None, None, None, None, None, None, dprelu)


# The CCBAM gate's input gradient, deferred (ccbam.py): its backward returns a stand-in of
# the input's shape (one element, expanded) and leaves the parts here, keyed by the stand-in's
# storage; the forked CBN backward that receives it forms the gradient inside its own passes
# (se_cbn_bwd_ccbam) instead of reading a written tensor.
_CCBAM_DX: dict = {}
CCBAM_DX_FUSED = [0]   # backward passes that took the deferred form (tests)


def ccbam_dx_defer(x, parts):
    """A stand-in gradient for x whose value is the CCBAM input gradient given by parts =
    (g, dP, idx, ca, dmean, dmax, amax) (se_ccbam_bwd_dx's operands)."""
    if len(_CCBAM_DX) > 64:   # stand-ins of graphs freed before their backward reached the CBN
        _CCBAM_DX.clear()
    tok = torch.empty(1, device=x.device, dtype=x.dtype).expand(x.shape)
    _CCBAM_DX[tok.data_ptr()] = (tok, parts)
    return tok


def _ccbam_dx_parts(g):
    if g is None or g.dim() == 0 or any(st != 0 for st in g.stride()):
        return None
    ent = _CCBAM_DX.get(g.data_ptr())
    if ent is None or ent[0].shape != g.shape:
        return None
    del _CCBAM_DX[g.data_ptr()]
    return ent[1]


def ccbam_dx_materialize(parts):
    """The deferred CCBAM input gradient written as a tensor (se_ccbam_bwd_dx)."""
    g, dP, idx, ca, dmean, dmax, amax = parts
    B, C = ca.shape
    dx = torch.empty_like(g)
    N.check(N.lib().se_ccbam_bwd_dx(g.data_ptr(), dP.data_ptr(), idx.data_ptr(), ca.data_ptr(), dmean.data_ptr(),
                                    dmax.data_ptr(), amax.data_ptr(), dx.data_ptr(), B, C, g[0, 0].numel(),
                                    N.stream_of(g)), "se_ccbam_bwd_dx")
    return dx


def complex_batch_norm(x, wrr, wri, wii, br, bi, running, nbt, training, eps, momentum,
                       act=ACT_NONE, slope=0.0, fork=False, prelu=None):
    """ComplexBatchNorm2d forward (+ optional fused activation) on the HIP path.
    running: (RMr, RMi, RVrr, RVri, RVii) or None; nbt: int64 tensor or None.
    prelu: the weight of a one-parameter nn.PReLU applied after the norm (fused).
    fork=True returns (y, alias of y) for two consumers: their two gradients are summed inside
    the backward kernels (se_cbn_bwd2) instead of by autograd's accumulation add."""
    out = _ComplexBN.apply(x, wrr, wri, wii, br, bi, running, nbt, training, eps, momentum,
                           act, slope, fork, prelu)
    if fork and isinstance(out, tuple):
        out[1]._sehip_cbn_fork = True   # a CCBAM gate reading it may defer its input gradient
    return out


class _FirstBlock(torch.autograd.Function):
    """A model's first block, conv -> ComplexBatchNorm2d + act, in training, with a
    conv input that needs no gradient (the noisy spectrum; FRCRN's encoder layer 0,
    frcrn.py:28-34, 62-76). Forward: the conv (exact fp32: the data-fed conv, see
    _pass_math) and the CBN forward. Backward: se_cbn_bwd_first_conv, the CBN
    backward with the conv's weight gradient accumulated in its apply pass (exact
    fp32 products), so the conv's dy is never written and no weight-grad GEMM reads
    it back. fork=True returns (y, alias of y) as complex_batch_norm."""

    @staticmethod
    def forward(ctx, x0, wr, wi, wrr, wri, wii, br, bi, running, nbt, eps, momentum, act, slope, cgeom, fork):
        kernel, stride, padding, padding_end, dilation = cgeom
        N.require_device(x0, wr, wi, wrr)
        x0 = x0.contiguous()
        lib = N.lib()
        out_channels = 2 * wr.shape[0]
        d = conv_desc(tuple(x0.shape), out_channels, kernel, stride, padding, dilation, (0, 0), False, True,
                      padding_end, exact=True)
        ho, wo = N.c_int(), N.c_int()
        N.check(lib.se_conv2d_out_shape(N.ctypes.byref(d), N.ctypes.byref(ho), N.ctypes.byref(wo)),
                "se_conv2d_out_shape")
        y0 = torch.empty((x0.shape[0], out_channels, ho.value, wo.value), device=x0.device, dtype=x0.dtype)
        ws = _workspace(lib.se_conv2d_workspace_size(N.ctypes.byref(d)), x0.device)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_conv2d_fwd(_with_math(d, "fwd"), x0.data_ptr(), wr.data_ptr(), wi.data_ptr(), None, None,
                                  y0.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_of(x0)), "se_conv2d_fwd")
        if t0 is not None:
            _TIMER.end(_gemm_tag("fwd", d), t0, _conv_flops(d), 4.0 * (x0.numel() + y0.numel() + 2 * wr.numel()))
        b, c = y0.shape[:2]
        hw = y0[0, 0].numel()
        y = torch.empty_like(y0)
        save = torch.empty(N.CBN_SAVE_FLOATS * (c // 2), device=x0.device, dtype=torch.float32)
        params = (wrr, wri, wii, br, bi)
        ws = _workspace(lib.se_cbn_workspace_size(b, c, hw), x0.device)
        ya = new_amax(x0.device)
        mom = -1.0 if momentum is None else float(momentum)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_cbn_fwd(y0.data_ptr(), y.data_ptr(), b, c, hw, N.ptr_array(params), N.ptr_array(running),
                               N.ptr(nbt), save.data_ptr(), 1, float(eps), mom, int(act), float(slope), ya.data_ptr(),
                               None, 0, ws.data_ptr(), ws.numel(), N.stream_of(x0)), "se_cbn_fwd")
        if t0 is not None:
            _TIMER.end("cbn_fwd", t0, 0.0, 4.0 * y0.numel() * 3)
        amax_put(y, ya)
        ctx.save_for_backward(x0, y0, save, wr, *params)
        ctx.cfg = (int(act), float(slope), d)
        if fork:
            ctx.set_materialize_grads(False)
            return y, y.view(y.shape)
        return y

    @staticmethod
    def backward(ctx, gy, gy2=None):
        x0, y0, save, wr, *params = ctx.saved_tensors
        act, slope, d = ctx.cfg
        if gy is None:
            gy, gy2 = gy2, None
        if gy is None:
            return (None,) * 16
        gy = gy.contiguous()
        gy2 = gy2.contiguous() if gy2 is not None else None
        b, c, h, w = y0.shape
        lib = N.lib()
        dwr, dwi = torch.empty_like(wr), torch.empty_like(wr)
        dparams = [torch.empty_like(p) for p in params]
        fc = N.FirstConvDesc()
        fc.x0, fc.cin, fc.in_h, fc.in_w = x0.data_ptr(), x0.shape[1] // 2, x0.shape[2], x0.shape[3]
        fc.kernel_h, fc.kernel_w, fc.stride_h, fc.stride_w = d.kernel_h, d.kernel_w, d.stride_h, d.stride_w
        fc.pad_h, fc.pad_w, fc.dil_h, fc.dil_w = d.pad_h, d.pad_w, d.dil_h, d.dil_w
        fc.dwr, fc.dwi = dwr.data_ptr(), dwi.data_ptr()
        ws = _workspace(lib.se_cbn_first_conv_workspace_size(b, c, h * w, fc.cin, fc.kernel_h, fc.kernel_w),
                        gy.device)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_cbn_bwd_first_conv(gy.data_ptr(), N.ptr(gy2), y0.data_ptr(), b, c, h, w,
                                          N.ptr_array(params), save.data_ptr(), N.ptr_array(dparams), 1, act, slope,
                                          N.ctypes.byref(fc), ws.data_ptr(), ws.numel(), N.stream_of(gy)),
                "se_cbn_bwd_first_conv")
        if t0 is not None:   # (gy [, gy2], y0) read twice, x0 taps from L2; no dx written
            _TIMER.end("cbn_bwd_first_conv", t0, _conv_flops(d), 4.0 * y0.numel() * (4 if gy2 is None else 6))
        return (None, dwr, dwi, *dparams, None, None, None, None, None, None, None, None)


def first_block_supported(x0, conv_w, bias, norm_training, kernel) -> bool:
    """The shapes se_cbn_bwd_first_conv covers: a training-mode first block on fp32
    CUDA tensors whose input carries no gradient, complex conv with one complex input
    channel, kernel (5, 2), no conv bias (SEHIP_FIRST_FUSED=0 turns it off)."""
    return (os.environ.get("SEHIP_FIRST_FUSED", "1") != "0" and norm_training and torch.is_grad_enabled()
            and x0.is_cuda and x0.dtype == torch.float32 and conv_w.dtype == torch.float32
            and not x0.requires_grad and bias is None and x0.shape[1] == 2 and tuple(kernel) == (5, 2))


def first_block(x0, wr, wi, wrr, wri, wii, br, bi, running, nbt, eps, momentum, act, slope, *, kernel, stride,
                padding, padding_end, dilation, fork=False):
    """act(CBN(conv(x0))) for a model's first block in training (see _FirstBlock)."""
    cgeom = (_pair(kernel), _pair(stride), _pair(padding), None if padding_end is None else _pair(padding_end),
             _pair(dilation))
    return _FirstBlock.apply(x0, wr, wi, wrr, wri, wii, br, bi, running, nbt, eps, momentum, act, slope, cgeom,
                             fork)


class _ComplexBNHead(torch.autograd.Function):
    """final_conv(act(CBN(x))) with final_conv = Conv2d(C, 2, (1, 2), bias=False):
    se_cbn_head_fwd / se_cbn_head_bwd (the activation y is never written)."""

    @staticmethod
    def forward(ctx, x, wrr, wri, wii, br, bi, w_head, running, nbt, training, eps, momentum, act, slope):
        N.require_device(x, wrr, w_head)
        x = x.contiguous()
        w_head = w_head.contiguous()
        b, c, h, w = x.shape
        out = torch.empty((b, w_head.shape[0], h, w - 1), device=x.device, dtype=x.dtype)
        save = torch.empty(N.CBN_SAVE_FLOATS * (c // 2), device=x.device, dtype=torch.float32)
        params = (wrr, wri, wii, br, bi) if wrr is not None else None
        lib = N.lib()
        ws = _workspace(lib.se_cbn_head_workspace_size(b, c, h * w), x.device)
        mom = -1.0 if momentum is None else float(momentum)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_cbn_head_fwd(x.data_ptr(), out.data_ptr(), b, c, h, w,
                                    N.ptr_array(params), N.ptr_array(running), N.ptr(nbt),
                                    save.data_ptr(), int(training), float(eps), mom, int(act),
                                    float(slope), w_head.data_ptr(), w_head.shape[0], w_head.shape[3],
                                    ws.data_ptr(), ws.numel(), N.stream_of(x)), "se_cbn_head_fwd")
        if t0 is not None:   # (1 read for the moments in training) + 1 read + write
            _TIMER.end("cbn_head_fwd", t0, 0.0, 4.0 * (x.numel() * (2 if training else 1) + out.numel()))
        ctx.save_for_backward(x, save, w_head, *(params or ()))
        ctx.cfg = (int(training), int(act), float(slope), params is not None)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, save, w_head, *params = ctx.saved_tensors
        training, act, slope, affine = ctx.cfg
        gout = gout.contiguous()
        b, c, h, w = x.shape
        dx = torch.empty_like(x)
        dw_head = torch.empty_like(w_head)
        dparams = [torch.empty_like(p) for p in params] if affine else None
        lib = N.lib()
        ws = _workspace(lib.se_cbn_head_workspace_size(b, c, h * w), x.device)
        dxa = new_amax(x.device) if training else None   # bound of max |dx| (the conv's dy)
        t0 = _TIMER.begin() if _TIMER else None
        N.check(lib.se_cbn_head_bwd(gout.data_ptr(), x.data_ptr(), dx.data_ptr(), b, c, h, w,
                                    N.ptr_array(params if affine else None), save.data_ptr(),
                                    N.ptr_array(dparams), w_head.data_ptr(), dw_head.data_ptr(),
                                    w_head.shape[0], w_head.shape[3], training, act, slope, N.ptr(dxa),
                                    ws.data_ptr(), ws.numel(), N.stream_of(gout)), "se_cbn_head_bwd")
        if dxa is not None:
            amax_put(dx, dxa)
        if t0 is not None:   # x read twice, dx written (the head gradient is L2-resident)
            _TIMER.end("cbn_head_bwd", t0, 0.0, 4.0 * (3 * x.numel() + 2 * gout.numel()))
        g = dparams or [None] * 5
        return (dx, *g, dw_head, None, None, None, None, None, None, None)


HEAD_SUPPORTED = ((2, 1, 2),)   # (out_channels, kernel_h, kernel_w) of se_cbn_head_*


def complex_batch_norm_head(x, wrr, wri, wii, br, bi, w_head, running, nbt, training, eps, momentum,
                            act=ACT_NONE, slope=0.0):
    """conv2d(act(ComplexBatchNorm2d(x)), w_head) for a real (1, 2)-kernel, 2-output,
    bias-free conv without padding (FRCRN's final_conv), fused: the activation is
    never written. Returns [B, 2, H, W - 1]."""
    return _ComplexBNHead.apply(x, wrr, wri, wii, br, bi, w_head, running, nbt, training, eps,
                                momentum, act, slope)


# --------------------------------------------------------------------------
# ConvSTFT / ConviSTFT — se_stft_* / se_istft_* (stft.hip)
# --------------------------------------------------------------------------
def stft_launch(x, out0, out1, window, twiddle, win, hop, nfft, center, mag_phase) -> None:
    """se_stft_fwd into preallocated outputs (the autograd Function's launch; bench bursts)."""
    b, length = x.shape
    N.check(N.lib().se_stft_fwd(x.data_ptr(), out0.data_ptr(), N.ptr(out1), b, length, win, hop, nfft,
                                int(center), int(mag_phase), window.data_ptr(), twiddle.data_ptr(),
                                N.dtype_code(x), N.stream_of(x)), "se_stft_fwd")


def istft_launch(spec, out, window, twiddle, win, hop, nfft, offset, out_len) -> None:
    """se_istft_fwd into a preallocated [B, out_len] output."""
    b, _, t = spec.shape
    N.check(N.lib().se_istft_fwd(spec.data_ptr(), out.data_ptr(), b, t, win, hop, nfft, offset, out_len,
                                 window.data_ptr(), twiddle.data_ptr(), N.dtype_code(spec),
                                 N.stream_of(spec)), "se_istft_fwd")


def istft_bwd_launch(gout, gspec, window, twiddle, win, hop, nfft, offset, out_len) -> None:
    """se_istft_bwd (the ConviSTFT adjoint) into a preallocated [B, nfft+2, T] gradient."""
    b, _, t = gspec.shape
    N.check(N.lib().se_istft_bwd(gout.data_ptr(), gspec.data_ptr(), b, t, win, hop, nfft, offset, out_len,
                                 window.data_ptr(), twiddle.data_ptr(), N.dtype_code(gout),
                                 N.stream_of(gout)), "se_istft_bwd")


class _Stft(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, window, twiddle, win, hop, nfft, center, mag_phase):
        N.require_device(window, twiddle)
        N.require_device(x, dtype=x.dtype)
        dt = N.dtype_code(x)
        x = x.contiguous()
        b, length = x.shape
        lib = N.lib()
        t = lib.se_stft_num_frames(length, win, hop, nfft, int(center))
        if t <= 0:
            raise RuntimeError(f"sehip ConvSTFT: input of length {length} too short for window {win}")
        half = nfft // 2 + 1
        if mag_phase:
            out0 = torch.empty((b, half, t), device=x.device, dtype=x.dtype)
            out1 = torch.empty_like(out0)
        else:
            out0 = torch.empty((b, 2 * half, t), device=x.device, dtype=x.dtype)
            out1 = None
        t0 = _TIMER.begin() if _TIMER else None
        stft_launch(x, out0, out1, window, twiddle, win, hop, nfft, center, mag_phase)
        if t0 is not None:   # algorithmic bytes: read the wav once, write the spectrum once
            _TIMER.end("stft_fwd", t0, 0.0, x.element_size() * (x.numel() + out0.numel()
                                                                 + (out1.numel() if mag_phase else 0)))
        return (out0, out1) if mag_phase else out0

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError("sehip ConvSTFT has no input gradient (the reference's basis "
                                  "is a fixed buffer and the training input carries no grad)")


def stft(x, window, twiddle, win, hop, nfft, center=True, mag_phase=False):
    """x: [B, L] -> spec [B, nfft+2, T] (or (mags, phase) [B, nfft/2+1, T])."""
    return _Stft.apply(x, window, twiddle, win, hop, nfft, center, mag_phase)


class _Istft(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, window, twiddle, win, hop, nfft, offset, out_len):
        N.require_device(window, twiddle)
        N.require_device(spec, dtype=spec.dtype)
        dt = N.dtype_code(spec)
        spec = spec.contiguous()
        b, rows, t = spec.shape
        if rows != nfft + 2:
            raise RuntimeError(f"sehip ConviSTFT: expected {nfft + 2} spectrum rows, got {rows}")
        out = torch.empty((b, out_len), device=spec.device, dtype=spec.dtype)
        t0 = _TIMER.begin() if _TIMER else None
        istft_launch(spec, out, window, twiddle, win, hop, nfft, offset, out_len)
        if t0 is not None:
            _TIMER.end("istft_fwd", t0, 0.0, spec.element_size() * (spec.numel() + out.numel()))
        ctx.save_for_backward(window, twiddle)
        ctx.cfg = (b, t, win, hop, nfft, offset, out_len)
        return out

    @staticmethod
    def backward(ctx, gout):
        window, twiddle = ctx.saved_tensors
        b, t, win, hop, nfft, offset, out_len = ctx.cfg
        gout = gout.contiguous()
        gspec = torch.empty((b, nfft + 2, t), device=gout.device, dtype=gout.dtype)
        t0 = _TIMER.begin() if _TIMER else None
        istft_bwd_launch(gout, gspec, window, twiddle, win, hop, nfft, offset, out_len)
        if t0 is not None:
            _TIMER.end("istft_bwd", t0, 0.0, gout.element_size() * (gout.numel() + gspec.numel()))
        return gspec, None, None, None, None, None, None, None


def istft(spec, window, twiddle, win, hop, nfft, offset, out_len):
    """spec [B, nfft+2, T] -> wav [B, out_len] = full OLA signal[offset:offset+out_len]."""
    return _Istft.apply(spec, window, twiddle, win, hop, nfft, offset, out_len)


class _Mask(torch.autograd.Function):
    """FRCRN's mask (frcrn.py:140-152) as one pass each way (se_mask_fwd / _bwd):
    est = pad(tanh(pad(h, top 1)) * spec[:, :, 1:], top 1) re-stacked [B, 2 half, T]."""

    @staticmethod
    def forward(ctx, h, spec, half):
        N.require_device(h, spec)
        h, spec = h.contiguous(), spec.contiguous()
        B, T = spec.shape[0], spec.shape[-1]
        if tuple(h.shape) != (B, 2, half - 2, T) or tuple(spec.shape) != (B, 2 * half, T):
            raise ValueError(f"sehip mask: h {tuple(h.shape)} / spec {tuple(spec.shape)} do not match half={half}")
        est = torch.empty_like(spec)
        N.check(N.lib().se_mask_fwd(h.data_ptr(), spec.data_ptr(), B, half, T, est.data_ptr(), N.stream_of(h)),
                "se_mask_fwd")
        ctx.save_for_backward(h, spec)
        ctx.half = half
        return est

    @staticmethod
    def backward(ctx, gest):
        h, spec = ctx.saved_tensors
        gest = gest.contiguous()
        gh = torch.empty_like(h)
        N.check(N.lib().se_mask_bwd(gest.data_ptr(), h.data_ptr(), spec.data_ptr(), spec.shape[0], ctx.half,
                                    spec.shape[-1], gh.data_ptr(), N.stream_of(gest)), "se_mask_bwd")
        return gh, None, None


POLAR_MASK_CALLS = [0]   # masks run by se_polar_mask_fwd (diagnostics / tests)


def _polar_planes_ok(ts):
    mr, mi, nr, ni = ts
    return (mr.is_cuda and mr.dtype in N.DTYPES and all(t.dtype == mr.dtype and t.device == mr.device for t in ts)
            and all(t.dim() == 3 and t.shape == mr.shape and t.stride(2) == 1 for t in ts)
            and mr.stride() == mi.stride() and nr.stride() == ni.stride())


def _polar_fwd(mr, mi, nr, ni, mode, row0=0):
    """row0: the mask's leading zero rows, not stored (mr / mi hold rows row0 .. F-1)."""
    B, Fq, T = nr.shape
    out = torch.empty((B, 2, Fq, T), device=nr.device, dtype=nr.dtype)
    N.check(N.lib().se_polar_mask_fwd(mr.data_ptr(), mi.data_ptr(), mr.stride(0), mr.stride(1), nr.data_ptr(),
                                      ni.data_ptr(), nr.stride(0), nr.stride(1), B, Fq, T, int(mode),
                                      N.dtype_code(nr), int(row0), out.data_ptr(), N.stream_of(nr)),
            "se_polar_mask_fwd")
    POLAR_MASK_CALLS[0] += 1
    return out


class _PolarMask(torch.autograd.Function):
    """DCCRN's 'E' mask (dccrn.py:194-207; or DCUNet's bounded_tanh, mode 0) as one pass each
    way (se_polar_mask_fwd / _bwd); the noisy planes take no gradient."""

    @staticmethod
    def forward(ctx, mr, mi, nr, ni, mode):
        ctx.save_for_backward(mr, mi, nr, ni)
        ctx.mode = mode
        return _polar_fwd(mr, mi, nr, ni, mode)

    @staticmethod
    def backward(ctx, g):
        mr, mi, nr, ni = ctx.saved_tensors
        g = g.contiguous()
        B, Fq, T = mr.shape
        dm = torch.empty((B, 2, Fq, T), device=g.device, dtype=g.dtype)
        N.check(N.lib().se_polar_mask_bwd(g.data_ptr(), mr.data_ptr(), mi.data_ptr(), mr.stride(0), mr.stride(1),
                                          nr.data_ptr(), ni.data_ptr(), nr.stride(0), nr.stride(1), B, Fq, T,
                                          int(ctx.mode), N.dtype_code(mr), 0, T, dm.data_ptr(), N.stream_of(g)),
                "se_polar_mask_bwd")
        return dm[:, 0], dm[:, 1], None, None, None


class _PolarMaskStored(torch.autograd.Function):
    """The mask taken from a stored decoder output m [B, 2, F - row0, Tm] (Tm >= T): mask row f
    is 0 for f < row0 (the reference's F.pad(m, (0, 0, row0, 0)), not materialised) and
    m[:, :, f - row0, :T] after (the trailing frames trimmed, dccrn.py:172-182). The backward
    writes m's gradient in m's own layout (0 on the trimmed frames) in the same pass."""

    @staticmethod
    def forward(ctx, m, nr, ni, mode, row0):
        ctx.save_for_backward(m, nr, ni)
        ctx.mode, ctx.row0 = mode, row0
        return _polar_fwd(m[:, 0], m[:, 1], nr, ni, mode, row0)

    @staticmethod
    def backward(ctx, g):
        m, nr, ni = ctx.saved_tensors
        g = g.contiguous()
        B, Fq, T = nr.shape
        dm = torch.empty_like(m)
        mr, mi = m[:, 0], m[:, 1]
        N.check(N.lib().se_polar_mask_bwd(g.data_ptr(), mr.data_ptr(), mi.data_ptr(), mr.stride(0), mr.stride(1),
                                          nr.data_ptr(), ni.data_ptr(), nr.stride(0), nr.stride(1), B, Fq, T,
                                          int(ctx.mode), N.dtype_code(m), int(ctx.row0), m.shape[3], dm.data_ptr(),
                                          N.stream_of(g)), "se_polar_mask_bwd")
        return dm, None, None, None, None


def polar_mask_stored(m, nr, ni, mode, row0=0):
    """polar_mask of the mask planes pad(m, top row0)[:, 0 / 1, :, :T] without the pad or the trim
    (_PolarMaskStored); None where the layout does not fit (m must be contiguous, of nr's dtype,
    with F - row0 rows and at least T frames) or the noisy planes need a gradient."""
    if not (m.is_cuda and m.dim() == 4 and m.shape[1] == 2 and m.is_contiguous() and m.dtype == nr.dtype
            and nr.dim() == 3 and m.shape[0] == nr.shape[0] and m.shape[2] + row0 == nr.shape[1]
            and m.shape[3] >= nr.shape[2] and nr.shape == ni.shape and nr.stride() == ni.stride()
            and nr.stride(2) == 1 and m.dtype in N.DTYPES):
        return None
    if torch.is_grad_enabled() and (nr.requires_grad or ni.requires_grad):
        return None
    if torch.is_grad_enabled() and m.requires_grad:
        return _PolarMaskStored.apply(m, nr, ni, int(mode), int(row0))
    return _polar_fwd(m[:, 0], m[:, 1], nr, ni, mode, row0)


def polar_mask(mr, mi, nr, ni, mode):
    """The magnitude / phase mask as a differentiable HIP op (_PolarMask): [B, 2, F, T], or
    None where the planes do not fit the kernels or the noisy planes need a gradient."""
    ts = (mr, mi, nr, ni)
    if not _polar_planes_ok(ts) or (torch.is_grad_enabled() and (nr.requires_grad or ni.requires_grad)):
        return None
    if torch.is_grad_enabled() and (mr.requires_grad or mi.requires_grad):
        return _PolarMask.apply(mr, mi, nr, ni, int(mode))
    return _polar_fwd(mr, mi, nr, ni, mode)


def polar_mask_nograd(mr, mi, nr, ni, mode):
    """The magnitude / phase masks of an inference forward in one pass (se_polar_mask_fwd):
    mode 0 DCUNet's bounded_tanh (dcunet.py:167-189), mode 1 DCCRN's 'E' (dccrn.py:194-207).
    mr / mi (mask) and nr / ni (noisy) are [B, F, T] planes, time contiguous. Returns
    [B, 2, F, T] (real, imaginary), or None where autograd needs the graph (a training
    forward keeps the reference's ops) or the planes do not fit the kernel's layout."""
    ts = (mr, mi, nr, ni)
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        return None
    if not _polar_planes_ok(ts):
        return None
    return _polar_fwd(mr, mi, nr, ni, mode)


def complex_mask(h, spec, half):
    """FRCRN's est spectrum from the final_conv output h [B, 2, half-2, T] and the
    ConvSTFT output spec [B, 2 half, T] (no gradient into spec)."""
    return _Mask.apply(h, spec.detach(), half)


# --------------------------------------------------------------------------
# LSTM layer of L stacked independent LSTMs — se_lstm_* (lstm.hip)
# --------------------------------------------------------------------------
_ZEROS: dict = {}


def _zero_row(n: int, device) -> torch.Tensor:
    key = (str(device), n)
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros(n, device=device, dtype=torch.float32)
    return z


def lstm_supported(hidden: int) -> bool:
    """H the HIP recurrence covers: 64 / 128 (se_lstm_*, one workgroup per
    sequence pair) and 256 / 512 / 1024 (se_lstm_wide_*, a group of H/32 or
    H/16 workgroups)."""
    return bool(N.lib().se_lstm_supported(int(hidden))) or bool(N.lib().se_lstm_wide_supported(int(hidden)))


_WIDE: dict = {}
_WIDE_PENDING: list = []   # (event, pinned status copy) of launched se_lstm_wide_* calls


def _wide_ws(device, stream: int):
    """(sync counters, status word) of se_lstm_wide_* for one (device, stream):
    a launch memsets its group counters and spins on them, so launches that may
    overlap (other streams) get their own. The status word stays 0 unless a
    group barrier timed out (the launch then wrote NaN; lstm_wide_poll raises)."""
    key = (str(device), int(stream))
    w = _WIDE.get(key)
    if w is None:
        n = int(N.lib().se_lstm_wide_sync_ints())
        w = _WIDE[key] = (torch.zeros(n, device=device, dtype=torch.int32),
                          torch.zeros(1, device=device, dtype=torch.int32))
    return w


def _wide_launched(status: torch.Tensor) -> None:
    """After a wide launch: a non-blocking copy of its status word to pinned host
    memory, checked by lstm_wide_poll once the launch has finished."""
    host = torch.empty(1, dtype=torch.int32, pin_memory=True)
    # the launch went to status.device's current stream (N.stream_of), which need not
    # be the current device's: copy and record on that stream
    stream = torch.cuda.current_stream(status.device)
    with torch.cuda.device(status.device), torch.cuda.stream(stream):
        host.copy_(status, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
    _WIDE_PENDING.append((ev, host))


class LstmWideTimeout(RuntimeError):
    """A se_lstm_wide_* group barrier timed out: not every workgroup of a group was
    resident at once (other work held the CUs), and the outputs are NaN."""


def lstm_wide_poll(block: bool = False) -> None:
    """Raise LstmWideTimeout if a finished se_lstm_wide_* launch reported a barrier
    timeout. Non-blocking by default (launches still running are checked later);
    block=True waits for all of them. Called before every wide launch and after
    every train_step, so a timeout surfaces within one step instead of as NaN."""
    keep = []
    for ev, host in _WIDE_PENDING:
        if block:
            ev.synchronize()
        if block or ev.query():
            if int(host[0]):
                _WIDE_PENDING.clear()
                raise LstmWideTimeout("sehip wide LSTM: a group barrier timed out (its workgroups were not all "
                                      "resident at once); the recurrence outputs are NaN")
        else:
            keep.append((ev, host))
    _WIDE_PENDING[:] = keep


def lstm_wide_status(device="cuda") -> int:
    """0 unless a se_lstm_wide_* group barrier timed out on `device` (on any
    stream; then its outputs were written as NaN). Synchronises."""
    dev = str(torch.device(device))
    return max([int(st.item()) for (d, _), (_, st) in _WIDE.items() if d == dev] or [0])


def _wide_check(rc: int, what: str, H: int) -> None:
    if rc == SE_E_UNSUPPORTED:
        raise RuntimeError(f"sehip {what}: hidden size {H} needs {H // (32 if H <= 512 else 16)} co-resident "
                           f"workgroups per group, more than this device's compute units allow")
    N.check(rc, what)


def _wide(H: int) -> bool:
    return H in (256, 512, 1024)


# --------------------------------------------------------------------------
# The LSTM layer GEMMs (input projection, input gradient, weight gradients, bias
# gradient) on se_gemm / se_colsum (csrc/gemm.hip: scaled split-fp16 MFMA, the
# conv GEMMs' f16x3 arithmetic) instead of torch.addmm / bmm on rocBLAS.
# SEHIP_LSTM_GEMM=torch runs them on torch (A/B measurement).
# --------------------------------------------------------------------------
_UNIT: dict = {}


def _unit_bound(dev) -> torch.Tensor:
    """fp32 [1] = 1.0: the bound of max |h| of an LSTM output (|o tanh(c)| < 1)."""
    t = _UNIT.get(dev)
    if t is None:
        t = _UNIT[dev] = torch.ones(1, device=dev)
    return t


def lstm_gemm_hip() -> bool:
    return os.environ.get("SEHIP_LSTM_GEMM", "hip") != "torch"


def gemm(A, B, C, *, M, N, K, lda, ldb, ldc, amax_a=None, amax_b=None, a_mcontig=False, b_ncontig=False,
         batches=1, sum_batches=False, stride_a=0, stride_b=0, stride_c=0, bias0=None, bias1=None, stride_bias=0,
         kmask=(0, 0), bias_rows=False, offsets=(0, 0, 0)):
    """C[b](m, n) = sum_k A(b, m, k) B(b, k, n) (+ bias0 + bias1) on se_gemm
    (include/sehip.h): A, B, C are device tensors of one storage type addressed from
    their data_ptr (+ offsets, in elements) with the given leading dimensions and batch
    strides. fp32: split-fp16 arithmetic scaled by amax_a / amax_b (bounds of max |A|,
    max |B|); bf16 / fp16: the one-term MFMA of that format (no bounds needed)."""
    nat = _NAT   # (N is the column count here)
    dt = nat.dtype_code(C)
    d = nat.GemmDesc(M=M, N=N, K=K, batches=batches, sum_batches=int(sum_batches), a_mcontig=int(a_mcontig),
                     b_ncontig=int(b_ncontig), lda=lda, ldb=ldb, ldc=ldc, stride_a=stride_a, stride_b=stride_b,
                     stride_c=stride_c, stride_bias=stride_bias, kmask_period=kmask[0], kmask_phase=kmask[1],
                     splits=0, dtype=dt, bias_rows=int(bias_rows))
    lib = nat.lib()
    es = C.element_size()
    ws = _workspace(lib.se_gemm_workspace_size(nat.ctypes.byref(d)), C.device)
    nat.check(lib.se_gemm(nat.ctypes.byref(d), A.data_ptr() + es * offsets[0], B.data_ptr() + es * offsets[1],
                          C.data_ptr() + es * offsets[2], nat.ptr(bias0), nat.ptr(bias1), nat.ptr(amax_a),
                          nat.ptr(amax_b), ws.data_ptr(), ws.numel(), nat.stream_of(C)), "se_gemm")
    return C


def _lstm_proj(x, w_ih, b_ih, b_hh, xa, wa):
    """x W_ih^T + b_ih + b_hh for L LSTMs: x [B, T, I] (shared) -> [B*T, L*G], or
    x [L, B, T, I] -> [L, B*T, G]."""
    L, G, I = w_ih.shape
    R = x.shape[-3] * x.shape[-2]
    if x.dim() == 3:
        out = torch.empty((R, L * G), device=x.device, dtype=torch.float32)
        return gemm(x, w_ih, out, M=R, N=L * G, K=I, lda=I, ldb=I, ldc=L * G, amax_a=xa, amax_b=wa,
                    bias0=b_ih, bias1=b_hh)
    out = torch.empty((L, R, G), device=x.device, dtype=torch.float32)
    return gemm(x, w_ih, out, M=R, N=G, K=I, lda=I, ldb=I, ldc=G, amax_a=xa, amax_b=wa, batches=L,
                stride_a=R * I, stride_b=G * I, stride_c=R * G, bias0=b_ih, bias1=b_hh, stride_bias=G)


def _lstm_grads_hip(ctx, x, w_ih, h, dg, xa, wa, need):
    """dx, dW_ih, dW_hh, db of _LstmLayer on se_gemm / se_colsum. dg [L, B*T, G]."""
    L, R, G = dg.shape
    I, H = w_ih.shape[2], h.shape[-1]
    T = h.shape[2]
    shared = x.dim() == 3
    dx = dw_ih = dw_hh = db = None
    if need[3]:   # the bias gradient pass also bounds max |dgates| (the GEMMs' scale)
        db = torch.empty((L, G), device=dg.device, dtype=torch.float32)
        ga = torch.empty(1, device=dg.device, dtype=torch.float32)
        lib = N.lib()
        ws = _workspace(lib.se_colsum_workspace_size(L, R, G), dg.device)
        N.check(lib.se_colsum(dg.data_ptr(), L, R, G, db.data_ptr(), ga.data_ptr(), ws.data_ptr(), ws.numel(),
                              N.stream_of(dg)), "se_colsum")
    else:
        ga = amax_of(dg)
    if need[0]:
        if shared:
            dx = torch.empty((x.shape[0], x.shape[1], I), device=dg.device, dtype=torch.float32)
            gemm(dg, w_ih, dx, M=R, N=I, K=G, lda=G, ldb=I, ldc=I, amax_a=ga, amax_b=wa, b_ncontig=True,
                 batches=L, sum_batches=True, stride_a=R * G, stride_b=G * I)
        else:
            dx = torch.empty_like(x)
            gemm(dg, w_ih, dx, M=R, N=I, K=G, lda=G, ldb=I, ldc=I, amax_a=ga, amax_b=wa, b_ncontig=True,
                 batches=L, stride_a=R * G, stride_b=G * I, stride_c=R * I)
    if need[1]:
        dw_ih = torch.empty_like(w_ih)
        gemm(dg, x, dw_ih, M=G, N=I, K=R, lda=G, ldb=I, ldc=I, amax_a=ga, amax_b=xa, a_mcontig=True,
             b_ncontig=True, batches=L, stride_a=R * G, stride_b=0 if shared else R * I, stride_c=G * I)
    if need[2]:
        dw_hh = torch.empty((L, G, H), device=dg.device, dtype=torch.float32)
        if T == 1 or R < 2:   # every h_{t-1} is h_{-1} = 0
            dw_hh.zero_()
        else:
            hf = h.reshape(L, R, H)
            hb = _unit_bound(dg.device)
            for rev in (0, 1):
                ls = [l for l in range(L) if ((ctx.rev_mask >> l) & 1) == rev]
                if not ls:
                    continue
                # forward: pairs (dgates row r, h row r - 1); reverse: (r, r + 1); the rows
                # of the first / last step of a sequence pair with nothing (k % T == T - 1)
                runs = [ls] if ls == list(range(ls[0], ls[0] + len(ls))) else [[l] for l in ls]
                for run in runs:
                    l0, n = run[0], len(run)
                    a = dg[l0, 1:] if rev == 0 else dg[l0, :-1]
                    b = hf[l0, :-1] if rev == 0 else hf[l0, 1:]
                    gemm(a, b, dw_hh[l0], M=G, N=H, K=R - 1, lda=G, ldb=H, ldc=H, amax_a=ga, amax_b=hb,
                         a_mcontig=True, b_ncontig=True, batches=n, stride_a=R * G, stride_b=R * H,
                         stride_c=G * H, kmask=(T, T - 1))
    return dx, dw_ih, dw_hh, db


def _bias_grads(ctx, db):
    """(d b_ih, d b_hh): both equal sum_t dgates_t, as separate tensors. Handing autograd
    the same tensor twice made the two parameters' .grad views of one buffer, which
    clip_grad_norm_'s in-place scaling then visited twice, racing (run-to-run differences
    in the LSTM biases, tools/determinism_probe.py)."""
    if db is None:
        return None, None
    both = ctx.has_b[0] and ctx.has_b[1]
    if both:
        from . import glue
        db2 = glue.copy_into(db, torch.empty_like(db))
    return (db if ctx.has_b[0] else None), ((db2 if both else db) if ctx.has_b[1] else None)


class _LstmLayer(torch.autograd.Function):
    """One layer of L independent LSTMs run together (torch.nn.LSTM math,
    gate order i, f, g, o, zero initial state).

    x: [B, T, I] fed to all L LSTMs, or [L, B, T, I]; w_ih [L, 4H, I];
    w_hh [L, 4H, H]; b_ih, b_hh [L, 4H] or None; bit l of rev_mask runs LSTM l
    right-to-left. Returns h [L, B, T, H].

    The input projection and all weight/input gradients are plain GEMMs on
    se_gemm (split-fp16 MFMA, csrc/gemm.hip; SEHIP_LSTM_GEMM=torch: rocBLAS
    through torch); the time recurrence is one persistent HIP launch per
    direction (fwd: se_lstm_fwd, bwd: se_lstm_bwd)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, rev_mask):
        N.require_device(x, w_ih, w_hh, b_ih, b_hh)
        L, G, I = w_ih.shape
        H = G // 4
        shared = x.dim() == 3
        B, T = x.shape[-3], x.shape[-2]
        if x.shape[-1] != I or tuple(w_hh.shape) != (L, G, H):
            raise ValueError("sehip lstm: inconsistent shapes")
        xa = wa = None
        x_lstm, x_row = (G, L * G) if shared else (B * T * G, G)
        if lstm_gemm_hip():   # se_gemm (csrc/gemm.hip)
            x, w_ih = x.contiguous(), w_ih.contiguous()
            b_ih = b_ih.contiguous() if b_ih is not None else None
            b_hh = b_hh.contiguous() if b_hh is not None else None
            xa, wa = amax_of(x), amax_of(w_ih)
            xproj = _lstm_proj(x, w_ih, b_ih, b_hh, xa, wa)
        else:                 # torch / rocBLAS (SEHIP_LSTM_GEMM=torch)
            bias = None
            if b_ih is not None or b_hh is not None:
                bias = (b_ih if b_ih is not None else 0) + (b_hh if b_hh is not None else 0)
            if shared:
                x2 = x.reshape(B * T, I)
                wt = w_ih.reshape(L * G, I).t()
                xproj = torch.addmm(bias.reshape(L * G), x2, wt) if bias is not None else x2 @ wt
            else:
                x3 = x.reshape(L, B * T, I)
                wt = w_ih.transpose(1, 2)
                xproj = (torch.baddbmm(bias.unsqueeze(1), x3, wt) if bias is not None
                         else torch.bmm(x3, wt))
        w_hh = w_hh.contiguous()
        h = torch.empty((L, B, T, H), device=x.device, dtype=x.dtype)
        c = torch.empty_like(h)
        gates = torch.empty((L, B, T, G), device=x.device, dtype=x.dtype)
        t0 = _TIMER.begin() if _TIMER else None
        if _wide(H):
            lstm_wide_poll()
            sync, status = _wide_ws(x.device, N.stream_of(x))
            _wide_check(N.lib().se_lstm_wide_fwd(xproj.data_ptr(), x_lstm, x_row, w_hh.data_ptr(), h.data_ptr(),
                                                 c.data_ptr(), gates.data_ptr(), L, B, T, H, int(rev_mask),
                                                 sync.data_ptr(), status.data_ptr(), N.stream_of(x)),
                        "se_lstm_wide_fwd", H)
            _wide_launched(status)
        else:
            N.check(N.lib().se_lstm_fwd(xproj.data_ptr(), x_lstm, x_row, w_hh.data_ptr(),
                                        _zero_row(H, x.device).data_ptr(), h.data_ptr(), c.data_ptr(),
                                        gates.data_ptr(), L, B, T, H, int(rev_mask), N.stream_of(x)),
                    "se_lstm_fwd")
        if t0 is not None:
            _TIMER.end("lstm_fwd", t0, 2.0 * L * B * T * G * H, 4.0 * L * B * T * (G + 2 * G + 2 * H))
        if xa is not None:
            amax_put(h, _unit_bound(h.device))   # |h| < 1: the next layer's input bound
        ctx.save_for_backward(x, w_ih, w_hh, h, c, gates)
        ctx.amax = (xa, wa)
        ctx.rev_mask, ctx.has_b = int(rev_mask), (b_ih is not None, b_hh is not None)
        ctx.mark_non_differentiable(c)
        ctx.set_materialize_grads(False)
        return h, c

    @staticmethod
    def backward(ctx, dh, dc):
        if dc is not None:
            raise NotImplementedError("sehip lstm: no gradient through the cell states (c_n)")
        x, w_ih, w_hh, h, c, gates = ctx.saved_tensors
        L, B, T, H = h.shape
        G, I = 4 * H, w_ih.shape[2]
        dh = torch.zeros_like(h) if dh is None else dh.contiguous()
        dgates = torch.empty_like(gates)
        t0 = _TIMER.begin() if _TIMER else None
        if _wide(H):
            lstm_wide_poll()
            sync, status = _wide_ws(dh.device, N.stream_of(dh))
            _wide_check(N.lib().se_lstm_wide_bwd(dh.data_ptr(), w_hh.data_ptr(), gates.data_ptr(), c.data_ptr(),
                                                 dgates.data_ptr(), L, B, T, H, ctx.rev_mask, sync.data_ptr(),
                                                 status.data_ptr(), N.stream_of(dh)),
                        "se_lstm_wide_bwd", H)
            _wide_launched(status)
        else:
            N.check(N.lib().se_lstm_bwd(dh.data_ptr(), w_hh.data_ptr(), gates.data_ptr(), c.data_ptr(),
                                        dgates.data_ptr(), L, B, T, H, ctx.rev_mask, N.stream_of(dh)),
                    "se_lstm_bwd")
        if t0 is not None:
            _TIMER.end("lstm_bwd", t0, 2.0 * L * B * T * G * H, 4.0 * L * B * T * (H + 2 * G + 2 * H))
        dg = dgates.reshape(L, B * T, G)
        shared = x.dim() == 3
        dx = dw_ih = dw_hh = db_ih = db_hh = None
        need_b = ctx.has_b[0] and ctx.needs_input_grad[3] or ctx.has_b[1] and ctx.needs_input_grad[4]
        if ctx.amax[0] is not None:   # the forward ran its projection on se_gemm
            need = (ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2], need_b)
            dx, dw_ih, dw_hh, db = _lstm_grads_hip(ctx, x, w_ih, h, dg, ctx.amax[0], ctx.amax[1], need)
            db_ih, db_hh = _bias_grads(ctx, db if need_b else None)
            return dx, dw_ih, dw_hh, db_ih, db_hh, None
        if ctx.needs_input_grad[0]:
            if shared:
                dx = torch.bmm(dg, w_ih).sum(0).reshape(B, T, I)
            else:
                dx = torch.bmm(dg, w_ih).reshape(L, B, T, I)
        if ctx.needs_input_grad[1]:
            xs = x.reshape(B * T, I) if shared else x.reshape(L, B * T, I)
            dw_ih = torch.stack([_tn_splitk(dg[l], xs if shared else xs[l]) for l in range(L)])
        if ctx.needs_input_grad[2]:
            # dW_hh[l] = sum_t dgates_t^T h_{t-1} (processing order; h_{-1} = 0), without
            # materialising the shifted h: on the flattened (b, t) rows the pairs are
            # (row r, row r - 1) forward / (r, r + 1) reverse, minus the B - 1 pairs that
            # straddle two sequences
            hf = h.reshape(L, B * T, H)
            dw_hh = torch.zeros((L, G, H), device=h.device, dtype=h.dtype)
            r = torch.arange(1, B, device=h.device) * T if B > 1 else None
            for l in (range(L) if T > 1 else ()):   # T = 1: every h_{t-1} is h_{-1} = 0
                if ((ctx.rev_mask >> l) & 1) == 0:
                    w = _tn_splitk(dg[l, 1:], hf[l, :-1])
                    if r is not None:   # rows b*T (t = 0) paired with the previous sequence's last h
                        w -= dg[l, r].t() @ hf[l, r - 1]
                else:
                    w = _tn_splitk(dg[l, :-1], hf[l, 1:])
                    if r is not None:   # rows b*T + T-1 (t = T-1) paired with the next sequence's first h
                        w -= dg[l, r - 1].t() @ hf[l, r]
                dw_hh[l] = w
        if need_b:
            db_ih, db_hh = _bias_grads(ctx, _rows_sum(dg))
        return dx, dw_ih, dw_hh, db_ih, db_hh, None


def _tn_splitk(a, b):
    """a^T b for row-major [R, G] and [R, I] (contiguous rows) with a long reduction
    R (the LSTM weight gradients, R = B*T): split-K over S row chunks (one bmm of S
    [G, I] products, summed in chunk order, plus the leftover rows), so the GEMM runs
    on S times the workgroups instead of a handful of long-K tiles."""
    R = a.shape[0]
    S = next((s for s in (32, 16, 8, 4, 2) if R // s >= 1024), 1)
    if S == 1:
        return a.t() @ b
    C = R // S
    out = torch.bmm(a[:S * C].view(S, C, -1).transpose(1, 2), b[:S * C].view(S, C, -1)).sum(0)
    if S * C < R:
        out += a[S * C:].t() @ b[S * C:]
    return out


def _rows_sum(a):
    """a.sum(1) for [L, R, G] with long R (the LSTM bias gradients): the rows in S
    chunks reduced first (S x more workgroups than ATen's reduction over R), then
    the S partial rows, in order."""
    L, R, G = a.shape
    S = next((s for s in (32, 16, 8, 4, 2) if R // s >= 1024), 1)
    if S == 1:
        return a.sum(1)
    C = R // S
    out = a[:, :S * C].reshape(L, S, C, G).sum(2).sum(1)
    if S * C < R:
        out += a[:, S * C:].sum(1)
    return out


def lstm_layer(x, w_ih, w_hh, b_ih=None, b_hh=None, rev_mask: int = 0, with_cell: bool = False):
    """h [L, B, T, H] of L stacked LSTMs over x ([B, T, I] shared or [L, B, T, I]);
    with_cell: (h, c) with the cell states c (no gradient through c)."""
    h, c = _LstmLayer.apply(x, w_ih, w_hh, b_ih, b_hh, rev_mask)
    return (h, c) if with_cell else h


# --------------------------------------------------------------------------
# Decoder skip join (frcrn.py:93-100 + complex_concat) — se_complex_join*
# --------------------------------------------------------------------------
class _ComplexJoin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        N.require_device(x, s, dtype=x.dtype)   # fp32, or bf16 / fp16 storage (bits copied)
        x, s = x.contiguous(), s.contiguous()
        B, Cx, Fx, Tx = x.shape
        _, Cs, Fs, Ts = s.shape
        out = torch.empty((B, Cx + Cs, Fs, Ts), device=x.device, dtype=x.dtype)
        N.check(N.lib().se_complex_join(x.data_ptr(), Cx, Fx, Tx, s.data_ptr(), Cs, Fs, Ts,
                                        out.data_ptr(), B, N.dtype_code(x), N.stream_of(x)), "se_complex_join")
        ctx.geom = (B, Cx, Fx, Tx, Cs, Fs, Ts)
        return out

    @staticmethod
    def backward(ctx, gout):
        B, Cx, Fx, Tx, Cs, Fs, Ts = ctx.geom
        gout = gout.contiguous()
        gx = torch.empty((B, Cx, Fx, Tx), device=gout.device, dtype=gout.dtype)
        gs = torch.empty((B, Cs, Fs, Ts), device=gout.device, dtype=gout.dtype)
        N.check(N.lib().se_complex_join_bwd(gout.data_ptr(), gx.data_ptr(), Cx, Fx, Tx, gs.data_ptr(),
                                            Cs, Fs, Ts, B, N.dtype_code(gout), N.stream_of(gout)),
                "se_complex_join_bwd")
        return gx, gs


def complex_join(x, skip):
    """complex_concat([align(x), skip]) where align crops x's trailing time
    columns / zero-pads its trailing frequency rows to skip's grid
    (frcrn.py:95-99), in one pass each way."""
    return _ComplexJoin.apply(x, skip)
