"""BatchNorm2d + activation on the HIP kernels (csrc/bn.hip): the
ConvBlock / ConvTransposeBlock body of CARN / GCARN (BatchNorm2d + PReLU,
models/_2104_05267_carn.py:30-56) and CRN (BatchNorm2d + ELU,
models/_1809_01405_crn.py:9-45). The modules stay nn.BatchNorm2d / nn.PReLU /
nn.ELU (constructor, parameters, buffers and state_dict keys unchanged);
``bn_act(norm, act, x)`` replaces ``act(norm(x))`` with one fused forward and
backward (training: batch statistics and the running-stat update as
nn.BatchNorm2d with a float momentum; eval: running statistics).
Configurations the kernels do not cover (momentum=None, non-4-D input, other
activations) run the modules themselves."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _native as N

_ACT_NONE, _ACT_PRELU, _ACT_ELU = 0, 1, 2


def _plane_stride(x):
    """Plane stride of a [B, C, H, W] tensor whose (b, c) planes are each HW
    contiguous floats at a constant stride (a row-cropped view qualifies)."""
    B, C, H, W = x.shape
    if x.stride(3) == 1 and x.stride(2) == W and x.stride(0) == C * x.stride(1) and x.stride(1) >= H * W:
        return x.stride(1)
    return None


class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act_param, rmean, rvar, training, momentum, eps, act, per_channel, alpha):
        # fp32, or bf16 / fp16 storage throughout (model.half() / .to(bfloat16)): read and
        # written in that dtype by the kernels, fp32 arithmetic
        N.require_device(x, weight, bias, act_param, rmean, rvar, dtype=x.dtype)
        dt = N.dtype_code(x)
        ps = _plane_stride(x)
        if ps is None:
            x = x.contiguous()
            ps = x.stride(1)
        B, C, H, W = x.shape
        y = torch.empty((B, C, H, W), device=x.device, dtype=x.dtype)
        save = torch.empty(2 * C, device=x.device, dtype=torch.float32)
        ws = torch.empty(int(N.lib().se_bn_workspace_size(B, C)), device=x.device, dtype=torch.uint8)
        N.check(N.lib().se_bn_fwd(x.data_ptr(), ps, B, C, H * W, N.ptr(weight), N.ptr(bias), N.ptr(rmean),
                                  N.ptr(rvar), int(training), float(momentum), float(eps), act, N.ptr(act_param),
                                  int(per_channel), float(alpha), y.data_ptr(), save.data_ptr(), dt, ws.data_ptr(),
                                  ws.numel(), N.stream_of(x)), "se_bn_fwd")
        ctx.save_for_backward(x, weight, bias, act_param, save)
        ctx.cfg = (ps, int(training), act, int(per_channel), float(alpha))
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, bias, act_param, save = ctx.saved_tensors
        ps, training, act, per_channel, alpha = ctx.cfg
        B, C, H, W = x.shape
        gy = gy.contiguous().to(x.dtype)
        dx = torch.empty((B, C, H, W), device=x.device, dtype=x.dtype)
        dw = torch.empty(C, device=x.device, dtype=x.dtype) if weight is not None else None
        db = torch.empty(C, device=x.device, dtype=x.dtype) if bias is not None else None
        da = torch.empty_like(act_param) if act_param is not None else None
        ws = torch.empty(int(N.lib().se_bn_workspace_size(B, C)), device=x.device, dtype=torch.uint8)
        N.check(N.lib().se_bn_bwd(gy.data_ptr(), x.data_ptr(), ps, B, C, H * W, N.ptr(weight), N.ptr(bias),
                                  save.data_ptr(), training, act, N.ptr(act_param), per_channel, alpha,
                                  dx.data_ptr(), N.ptr(dw), N.ptr(db), N.ptr(da), N.dtype_code(x), ws.data_ptr(),
                                  ws.numel(), N.stream_of(gy)), "se_bn_bwd")
        return dx, dw, db, da, None, None, None, None, None, None, None, None


def bn_act(norm: nn.Module, act: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """act(norm(x)) for nn.BatchNorm2d / nn.Identity `norm` and nn.PReLU / nn.ELU /
    nn.Identity `act`, fused on the HIP kernels when norm is a BatchNorm2d."""
    if not isinstance(norm, nn.BatchNorm2d) or not x.is_cuda or x.dim() != 4:
        return act(norm(x))
    if isinstance(act, nn.PReLU):
        code, param, alpha = _ACT_PRELU, act.weight, 0.0
    elif isinstance(act, nn.ELU) and not act.inplace:
        code, param, alpha = _ACT_ELU, None, float(act.alpha)
    elif isinstance(act, nn.Identity):
        code, param, alpha = _ACT_NONE, None, 0.0
    else:
        return act(norm(x))
    use_batch = norm.training or not norm.track_running_stats
    if norm.momentum is None and norm.training and norm.track_running_stats:
        return act(norm(x))     # cumulative average: needs the step count on the host
    if not use_batch and norm.running_mean is None:
        return act(norm(x))
    track = norm.training and norm.track_running_stats
    rmean = norm.running_mean if (track or not use_batch) else None
    rvar = norm.running_var if (track or not use_batch) else None
    if x.dtype not in N.DTYPES or any(t is not None and t.dtype != x.dtype
                                      for t in (norm.weight, norm.bias, param, rmean, rvar)):
        return act(norm(x))     # mixed dtypes: the modules themselves
    if track:
        norm.num_batches_tracked.add_(1)
    return _BnAct.apply(x, norm.weight, norm.bias, param, rmean, rvar, use_batch, norm.momentum or 0.0, norm.eps,
                        code, param is not None and param.numel() > 1, alpha)
