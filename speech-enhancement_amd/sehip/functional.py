"""Autograd functions over the sehip C ABI (include/sehip.h).

Each Function validates shapes on the host, allocates outputs and workspace
through PyTorch's caching allocator, and launches on the caller's current
HIP stream. There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import torch

from . import _native as N


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# --------------------------------------------------------------------------
# Complex / real (transposed) conv2d — se_conv2d_* (cconv.hip)
# --------------------------------------------------------------------------
def conv_desc(x_shape, out_channels, kernel, stride, padding, dilation, output_padding,
              transposed, complex_w) -> N.ConvDesc:
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
    return d


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wr, wi, br, bi, geom):
        out_channels, kernel, stride, padding, dilation, output_padding, transposed, complex_w = geom
        N.require_device(x, wr, wi, br, bi)
        x = x.contiguous()
        d = conv_desc(tuple(x.shape), out_channels, kernel, stride, padding, dilation,
                      output_padding, transposed, complex_w)
        lib = N.lib()
        ho, wo = N.c_int(), N.c_int()
        N.check(lib.se_conv2d_out_shape(N.ctypes.byref(d), N.ctypes.byref(ho), N.ctypes.byref(wo)),
                "se_conv2d_out_shape")
        y = torch.empty((x.shape[0], out_channels, ho.value, wo.value), device=x.device, dtype=x.dtype)
        nbytes = lib.se_conv2d_workspace_size(N.ctypes.byref(d))
        ws = _workspace(nbytes, x.device)
        N.check(lib.se_conv2d_fwd(N.ctypes.byref(d), x.data_ptr(), wr.data_ptr(), N.ptr(wi),
                                  N.ptr(br), N.ptr(bi), y.data_ptr(), ws.data_ptr(), ws.numel(),
                                  N.stream_of(x)), "se_conv2d_fwd")
        ctx.save_for_backward(x, wr, wi)
        ctx.desc, ctx.nbytes, ctx.has_bias = d, nbytes, br is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wr, wi = ctx.saved_tensors
        gy = gy.contiguous()
        d, lib = ctx.desc, N.lib()
        ws = _workspace(ctx.nbytes, gy.device)
        dx = dwr = dwi = dbr = dbi = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            N.check(lib.se_conv2d_bwd_data(N.ctypes.byref(d), gy.data_ptr(), wr.data_ptr(), N.ptr(wi),
                                           dx.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_of(gy)),
                    "se_conv2d_bwd_data")
        if any(ctx.needs_input_grad[1:5]):
            dwr = torch.empty_like(wr)
            dwi = torch.empty_like(wi) if wi is not None else None
            if ctx.has_bias:
                nb = d.out_channels // 2 if d.complex_weights else d.out_channels
                dbr = torch.empty(nb, device=gy.device, dtype=gy.dtype)
                dbi = torch.empty(nb, device=gy.device, dtype=gy.dtype) if d.complex_weights else None
            N.check(lib.se_conv2d_bwd_weight(N.ctypes.byref(d), x.data_ptr(), gy.data_ptr(),
                                             dwr.data_ptr(), N.ptr(dwi), N.ptr(dbr), N.ptr(dbi),
                                             ws.data_ptr(), ws.numel(), N.stream_of(gy)),
                    "se_conv2d_bwd_weight")
        return dx, dwr, dwi, dbr, dbi, None


def conv2d(x, wr, wi=None, br=None, bi=None, *, out_channels, kernel, stride=1, padding=0,
           dilation=1, output_padding=0, transposed=False):
    """Fused complex conv (wi given) or real conv (wi None) on the HIP path."""
    geom = (int(out_channels), _pair(kernel), _pair(stride), _pair(padding), _pair(dilation),
            _pair(output_padding), bool(transposed), wi is not None)
    return _Conv2d.apply(x, wr, wi, br, bi, geom)
