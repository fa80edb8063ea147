"""Parameter update of the train step on the HIP kernels (csrc/step.hip):
torch.nn.utils.clip_grad_norm_ and torch.optim.AdamW (trainer.py:216-221,
hparams: AdamW, clip 0.5) over a device table of parameter slots, so a step
is three launches (sum of squares, clip, AdamW) whatever the tensor count.

Drop-in surface: ``AdamW`` takes torch.optim.AdamW's arguments (amsgrad,
maximize, capturable, differentiable off) and keeps its state layout
(state[p] = {'step', 'exp_avg', 'exp_avg_sq'}), so state_dicts load either way;
``clip_grad_norm_`` has torch's signature for the 2-norm and returns the
total norm as a device tensor. Both need contiguous CUDA tensors of one
storage type per call: fp32, or the bf16 / fp16 of a model.to(bfloat16) /
.half() run (ABI 10: torch's foreach AdamW rounding reproduced in the kernel).
There is no CPU path.
"""
from __future__ import annotations


import numpy as np
import torch

from . import _native as N

SUMSQ_DOUBLES = 2049   # SE_SUMSQ_DOUBLES (include/sehip.h)
_SLOT = np.dtype([("param", "<u8"), ("grad", "<u8"), ("exp_avg", "<u8"), ("exp_avg_sq", "<u8"),
                  ("numel", "<i8"), ("offset", "<i8")])


def _slot_table(rows, device):
    """Device array of se_tensor_slot for [(param, grad, exp_avg, exp_avg_sq)]
    (None -> NULL). Returns (table, nslots, total)."""
    arr = np.zeros(len(rows), dtype=_SLOT)
    off = 0
    for i, (p, g, m, v) in enumerate(rows):
        n = g.numel()
        arr[i] = (N.ptr(p) or 0, g.data_ptr(), N.ptr(m) or 0, N.ptr(v) or 0, n, off)
        off += n
    host = torch.from_numpy(arr.view(np.uint8)).pin_memory()
    return host.to(device, non_blocking=True), len(rows), off


def _check(ts):
    """The storage-type code (SE_DTYPE_*) shared by every tensor, or RuntimeError."""
    dt = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda or t.dtype not in N.DTYPES or not t.is_contiguous() or (dt is not None and t.dtype != dt):
            raise RuntimeError("sehip optim: parameters and gradients must be contiguous CUDA tensors of one "
                               "storage type (fp32, bf16 or fp16; there is no CPU path)")
        dt = t.dtype
    return N.DTYPES[dt] if dt is not None else 0


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False, foreach=None):
    """torch.nn.utils.clip_grad_norm_ (2-norm): scales every .grad in place by
    min(max_norm / (total_norm + 1e-6), 1) and returns total_norm (device fp32).
    Sum of squares in fp64 (torch: fp32 per-tensor norms)."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("sehip clip_grad_norm_: only the 2-norm (the reference's)")
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    code = _check(grads)
    dev = grads[0].device
    table, n, total = _slot_table([(None, g, None, None) for g in grads], dev)
    sumsq = torch.empty(SUMSQ_DOUBLES, device=dev, dtype=torch.float64)
    norm = torch.empty(1, device=dev, dtype=torch.float32)
    st = N.stream_of(grads[0])
    N.check(N.lib().se_grad_sumsq(table.data_ptr(), n, total, sumsq.data_ptr(), code, st), "se_grad_sumsq")
    if error_if_nonfinite and not torch.isfinite(sumsq[0]).item():   # [0] = the total (SE_SUMSQ_DOUBLES)
        raise RuntimeError(f"The total norm of order {float(norm_type)} for gradients from `parameters` "
                           "is non-finite, so it cannot be clipped")
    N.check(N.lib().se_clip_grads(table.data_ptr(), n, total, sumsq.data_ptr(), float(max_norm), norm.data_ptr(),
                                  code, st), "se_clip_grads")
    return norm.view(())


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW on se_adamw_step: one launch per (parameter group, step
    count). Parameters of a group normally share their step count; one that
    missed steps (no gradient on some iterations, or a loaded state_dict with
    per-parameter steps) is updated by its own launch with its own bias
    corrections, as torch tracks the step per parameter."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 *, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("sehip AdamW: amsgrad / maximize / capturable / differentiable")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_step: dict = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("sehip AdamW: sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                s = int(st["step"].item())   # a CPU tensor, as torch's non-capturable AdamW
                by_step.setdefault(s, []).append((p, p.grad, st["exp_avg"], st["exp_avg_sq"]))
            b1, b2 = group["betas"]
            for step_val, rows in sorted(by_step.items()):
                by_dtype: dict = {}
                for r in rows:
                    by_dtype.setdefault(r[0].dtype, []).append(r)
                for rs in by_dtype.values():
                    code = _check([t for r in rs for t in r])
                    table, n, total = _slot_table(rs, rs[0][0].device)
                    N.check(N.lib().se_adamw_step(table.data_ptr(), n, total, float(group["lr"]), float(b1),
                                                  float(b2), float(group["eps"]), float(group["weight_decay"]),
                                                  step_val, code, N.stream_of(rs[0][0])), "se_adamw_step")
        return loss
