"""Complex CBAM skip attention (FRCRN decoder), HIP path.

Drop-in for models/modules/ccbam.py (same module tree and state_dict keys).
CCBAM.forward runs the fused path (_CCBAMFn): the five passes over the full
skip tensor are csrc/ccbam.hip kernels (se_ccbam_*), the shared MLP and the
spatial ComplexConv2d(4->2, k7) + CBN + ReLU run as their own modules on the
small pooled maps (the conv/CBN on the HIP conv and CBN kernels). The
sub-modules' own forward methods (ChannelAttention, SpatialAttention) keep
the unfused reference formulation for anyone calling them directly.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import _native as N
from . import functional as F
from .complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexLinear, complex_concat,
                         merge_real_imag, norm_act, split_complex)


class ConvBlock(nn.Module):
    """ccbam.py:7-16."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, **kwargs):
        super().__init__()
        self.conv = ComplexConv2d(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = ComplexBatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return norm_act(self.norm, self.act, self.conv(x))


class LinearBlock(nn.Module):
    """ccbam.py:18-26."""

    def __init__(self, in_channels, out_channels, act=True, **kwargs):
        super().__init__()
        self.linear = ComplexLinear(in_channels, out_channels, **kwargs)
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return self.act(self.linear(x))


class ChannelAttention(nn.Module):
    """ccbam.py:28-63. The avg- and max-pooled descriptors go through the
    shared MLP as one stacked batch (same weights, one GEMM per layer)."""

    def __init__(self, feature_map_channels, r=16):
        super().__init__()
        reduction = feature_map_channels // r if feature_map_channels // r else 2
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.max_pool = nn.AdaptiveMaxPool2d((1, 1))
        self.shared_fc_layer = nn.Sequential(
            LinearBlock(feature_map_channels, reduction, act=True, bias=False),
            LinearBlock(reduction, feature_map_channels, act=False, bias=False))

    def forward(self, x):
        b, c = x.shape[:2]
        pooled = torch.cat([x.mean(dim=(2, 3)), x.amax(dim=(2, 3))], dim=0)
        a, m = torch.chunk(self.shared_fc_layer(pooled), 2, dim=0)
        return torch.sigmoid(a + m).view(b, c, 1, 1)


class SpatialAttention(nn.Module):
    """ccbam.py:65-86."""

    def __init__(self):
        super().__init__()
        self.conv = ConvBlock(in_channels=4, out_channels=2, kernel_size=7, padding=3)

    def forward(self, x):
        re, im = split_complex(x)
        avg = torch.cat([re.mean(1, keepdim=True), im.mean(1, keepdim=True)], dim=1)
        mx = torch.cat([re.amax(1, keepdim=True), im.amax(1, keepdim=True)], dim=1)
        return torch.sigmoid(self.conv(complex_concat([avg, mx], dim=1)))


def _call(fn, name, *args):
    N.check(fn(*args), name)


def _mlp_weights(cab: "ChannelAttention", B: int, C: int):
    """(w1r, w1i, w2r, w2i) when the channel branch's MLP is the reference's
    (ComplexLinear(C, Hd, bias=False) -> ReLU -> ComplexLinear(Hd, C, bias=False),
    ccbam.py:36-39) on fp32 tensors and fits se_ccbam_mlp_*; else None (the MLP then
    runs as its own modules). SEHIP_CCBAM_MLP=0 turns the fused kernels off."""
    if os.environ.get("SEHIP_CCBAM_MLP", "1") == "0":
        return None
    fc = cab.shared_fc_layer
    if len(fc) != 2 or not all(isinstance(b, LinearBlock) for b in fc):
        return None
    l1, l2 = fc[0].linear, fc[1].linear
    if not (isinstance(fc[0].act, nn.ReLU) and isinstance(fc[1].act, nn.Identity)):
        return None
    ws = (l1.real_linear.weight, l1.imag_linear.weight, l2.real_linear.weight, l2.imag_linear.weight)
    if any(lin.bias is not None for lin in (l1.real_linear, l1.imag_linear, l2.real_linear, l2.imag_linear)):
        return None
    if any(w.dtype != torch.float32 or not w.is_cuda or not w.is_contiguous() for w in ws):
        return None
    Hd = 2 * ws[0].shape[0]
    if ws[0].shape[1] * 2 != C or tuple(ws[2].shape) != (C // 2, Hd // 2) or (B * C + 2 * B * Hd) * 4 > 64 * 1024:
        return None
    return ws


class _CCBAMFn(torch.autograd.Function):
    """out = CCBAM(x) with the full-tensor passes on se_ccbam_* kernels.

    The MLP (channel branch) and conv/CBN/ReLU (spatial branch) are built as
    small autograd graphs inside forward (on detached pooled inputs) and
    differentiated with torch.autograd.grad in backward, so their parameters
    (and CBN's HIP kernels) are used unchanged."""

    @staticmethod
    def forward(ctx, x, mod, *params):
        N.require_device(x)
        x = x.contiguous()
        t0 = F._TIMER.begin() if F._TIMER else None
        B, C, H, W = x.shape
        HW = H * W
        lib, st, dev = N.lib(), N.stream_of(x), x.device
        need_grad = any(ctx.needs_input_grad)
        # SEHIP_CCBAM_DEFER_DX=1 and the input a forked ComplexBatchNorm2d output (FRCRN's
        # encoder skip): the input gradient is left to that CBN's backward to form
        # (se_cbn_bwd_ccbam), never written here. Two skip-sized passes fewer per gate, but the
        # main-stream CBN backward grows by what the side stream saves: the step measured
        # neutral (-0.3 %, profiles/ab/r6_ccbam_defer_dx_ab.log), so it is off by default.
        ctx.defer_dx = bool(getattr(x, "_sehip_cbn_fork", False)) and x.dtype == torch.float32 and \
            os.environ.get("SEHIP_CCBAM_DEFER_DX", "0") == "1"
        cab, sab = mod.channel_attention_branch, mod.spatial_attention_branch
        mean = torch.empty(B, C, device=dev)
        mx = torch.empty(B, C, device=dev)
        amax = torch.empty(B, C, device=dev, dtype=torch.int32)
        _call(lib.se_ccbam_channel_pool, "se_ccbam_channel_pool", x.data_ptr(), mean.data_ptr(),
              mx.data_ptr(), amax.data_ptr(), B, C, HW, st)
        mlp = _mlp_weights(cab, B, C)
        pooled = hs = None
        if mlp is not None:   # the whole MLP + sigmoid in one launch (se_ccbam_mlp_fwd)
            ca = torch.empty(B, C, device=dev)
            hs = torch.empty(2 * B, 2 * mlp[0].shape[0], device=dev)
            _call(lib.se_ccbam_mlp_fwd, "se_ccbam_mlp_fwd", mean.data_ptr(), mx.data_ptr(),
                  *(w.data_ptr() for w in mlp), B, C, hs.shape[1], ca.data_ptr(), hs.data_ptr(), st)
        else:
            with torch.set_grad_enabled(need_grad):
                pooled = torch.cat([mean, mx], 0)
                if need_grad:
                    pooled.requires_grad_(True)
                a, m = torch.chunk(cab.shared_fc_layer(pooled), 2, dim=0)
                ca = torch.sigmoid(a + m).contiguous()               # [B, C]
        P = torch.empty(B, 4, H, W, device=dev)
        idx = torch.empty(B, 2, H, W, device=dev, dtype=torch.int16)
        _call(lib.se_ccbam_spatial_pool, "se_ccbam_spatial_pool", x.data_ptr(), ca.data_ptr(),
              P.data_ptr(), idx.data_ptr(), B, C, HW, st)
        with torch.set_grad_enabled(need_grad):
            Pl = P.requires_grad_(True) if need_grad else P
            z = sab.conv(Pl)                                          # [B, 2, H, W] pre-sigmoid
        # the gate's sigmoid outside autograd: its backward is fused into
        # se_ccbam_bwd_sa_sigmoid
        zc = z.detach().contiguous()
        sa = torch.empty_like(zc)
        _call(lib.se_sigmoid_fwd, "se_sigmoid_fwd", zc.data_ptr(), sa.data_ptr(), zc.numel(), 0, st)
        out = torch.empty_like(x)
        oa = F.new_amax(dev)   # max |out|, found by the apply pass: the consumers' F16X3 scale source
        _call(lib.se_ccbam_apply, "se_ccbam_apply", x.data_ptr(), ca.data_ptr(), sa.data_ptr(),
              out.data_ptr(), B, C, HW, oa.data_ptr(), st)
        F.amax_put(out, oa)
        if t0 is not None:   # algorithmic bytes: x read once, out written once
            F._TIMER.end("ccbam_fwd", t0, 0.0, 2.0 * x.numel() * x.element_size())
        if need_grad:
            ctx.save_for_backward(x, idx, amax)
            ctx.graphs = (pooled, ca, Pl, z, sa)
            ctx.mod = mod
            ctx.mlp = (mlp, mean, mx, hs) if mlp is not None else None
        return out

    @staticmethod
    def backward(ctx, gout):
        x, idx, amax = ctx.saved_tensors
        pooled, ca, Pl, z, sa = ctx.graphs
        mod = ctx.mod
        B, C, H, W = x.shape
        HW = H * W
        lib, st, dev = N.lib(), N.stream_of(gout), gout.device
        gout = gout.contiguous()
        t0 = F._TIMER.begin() if F._TIMER else None
        dz = torch.empty(B, 2, H, W, device=dev)   # d loss / d (pre-sigmoid gate)
        _call(lib.se_ccbam_bwd_sa_sigmoid, "se_ccbam_bwd_sa_sigmoid", gout.data_ptr(), sa.data_ptr(),
              dz.data_ptr(), B, C, HW, st)
        sp = list(mod.spatial_attention_branch.parameters())
        ch = list(mod.channel_attention_branch.parameters())
        gs = torch.autograd.grad(z, [Pl] + sp, dz, allow_unused=True)
        dP = gs[0].contiguous()
        dca = torch.empty(B, C, device=dev)
        ws = F._workspace(lib.se_ccbam_workspace_size(B, C, HW), dev)
        _call(lib.se_ccbam_bwd_dca, "se_ccbam_bwd_dca", gout.data_ptr(), x.data_ptr(), dP.data_ptr(),
              idx.data_ptr(), dca.data_ptr(), B, C, HW, ws.data_ptr(), ws.numel(), st)
        if ctx.mlp is not None:   # se_ccbam_mlp_bwd: dmean, dmax and the four weight gradients
            mlp, mean, mx, hs = ctx.mlp
            dmean, dmax = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
            dws = [torch.empty_like(w) for w in mlp]
            _call(lib.se_ccbam_mlp_bwd, "se_ccbam_mlp_bwd", dca.data_ptr(), ca.data_ptr(), mean.data_ptr(),
                  mx.data_ptr(), hs.data_ptr(), *(w.data_ptr() for w in mlp), B, C, hs.shape[1],
                  dmean.data_ptr(), dmax.data_ptr(), *(d.data_ptr() for d in dws), st)
            by_id = {id(w): d for w, d in zip(mlp, dws)}
            gc = [None] + [by_id.get(id(p)) for p in ch]
            ctx.mlp = None
        else:
            gc = torch.autograd.grad(ca, [pooled] + ch, dca, allow_unused=True)
            dmean, dmax = (t.contiguous() for t in torch.chunk(gc[0], 2, dim=0))
        if ctx.defer_dx:   # formed inside the forked CBN's backward (functional.ccbam_dx_defer)
            dx = F.ccbam_dx_defer(x, (gout, dP, idx, ca, dmean, dmax, amax))
        else:
            dx = torch.empty_like(x)
            _call(lib.se_ccbam_bwd_dx, "se_ccbam_bwd_dx", gout.data_ptr(), dP.data_ptr(), idx.data_ptr(),
                  ca.data_ptr(), dmean.data_ptr(), dmax.data_ptr(), amax.data_ptr(), dx.data_ptr(),
                  B, C, HW, st)
        if t0 is not None:   # algorithmic bytes: gout and x read once (+ dx written once)
            F._TIMER.end("ccbam_bwd", t0, 0.0, (2.0 if ctx.defer_dx else 3.0) * x.numel() * x.element_size())
        grads = {id(p): g for p, g in zip(sp, gs[1:])}
        grads.update({id(p): g for p, g in zip(ch, gc[1:])})
        del ctx.graphs
        return (dx, None) + tuple(grads.get(id(p)) for p in mod.parameters())


class CCBAM(nn.Module):
    """ccbam.py:88-106: channel gate (multiplicative), then the 2-channel
    spatial map ADDED to the real and the imaginary halves (fused: _CCBAMFn)."""

    def __init__(self, feature_map_channels, reduction=16):
        super().__init__()
        self.channel_attention_branch = ChannelAttention(feature_map_channels, reduction)
        self.spatial_attention_branch = SpatialAttention()

    def forward(self, x):
        return _CCBAMFn.apply(x, self, *self.parameters())

    def forward_unfused(self, x):
        """The reference's op-by-op formulation (PyTorch device ops)."""
        x = x * self.channel_attention_branch(x)
        sa = self.spatial_attention_branch(x)
        re, im = split_complex(x)
        return merge_real_imag(x, re + sa[:, 0:1], im + sa[:, 1:2], dim=1)
