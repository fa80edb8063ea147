"""Training step and data-parallel launcher.

``train_step`` reproduces one iteration of the reference hot loop
(trainer.py:99-124 + _update_parameters at :210-221): model -> mono ->
pad/truncate -> SI-SNR -> backward -> clip_grad_norm_(0.5) -> AdamW.step ->
zero_grad. The reference's DDP path never worked (no init_process_group,
multi-element device_ids); ``setup_distributed`` builds the
real one: one process per GPU, torch.distributed over RCCL ("nccl" is RCCL
on ROCm), DistributedDataParallel bucketing the 7.7 MB gradient all-reduce
over xGMI during backward. ComplexBatchNorm keeps per-rank statistics like
nn.BatchNorm2d under DDP (the reference has no SyncBN).
"""
from __future__ import annotations

import os

import torch

from .losses import SI_SNR_loss, pad_or_truncate_wav, reshape_wav_to_mono

ADAMW = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)   # hparams/*.py
CLIP_NORM = 0.5                                                           # hyperparams.py:10


def make_optimizer(model, **overrides):
    kw = dict(ADAMW)
    kw.update(overrides)
    return torch.optim.AdamW(model.parameters(), **kw)


def _defer_ok(model) -> bool:
    """Deferred weight-grads (functional.deferred_weight_grads) need every .grad
    None on entry and no gradient hooks during backward: not under DDP, and
    only on the GPU."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return False
    p = next(model.parameters(), None)
    return p is not None and p.is_cuda and all(q.grad is None for q in model.parameters()) \
        and os.environ.get("SEHIP_OVERLAP", "1") != "0"


_MAIN_STREAMS: dict = {}


def _main_stream(device):
    """SEHIP_MAIN_PRIO (e.g. -1): run the step on a stream of that HIP priority, so the
    command processor dispatches its (critical-path) workgroups ahead of the
    deferred weight-grad side stream's when CUs free up. None = the current stream."""
    prio = int(os.environ.get("SEHIP_MAIN_PRIO", "0"))
    if not prio or device.type != "cuda":
        return None
    s = _MAIN_STREAMS.get(device)
    if s is None:
        s = _MAIN_STREAMS[device] = torch.cuda.Stream(device, priority=prio)
    return s


def train_step(model, optimizer, noisy, clean, clip_norm=CLIP_NORM):
    """One optimisation step; returns the (device) loss, no host sync."""
    hp = _main_stream(noisy.device)
    if hp is None:
        return _train_step(model, optimizer, noisy, clean, clip_norm)
    cur = torch.cuda.current_stream(noisy.device)
    hp.wait_stream(cur)
    with torch.cuda.stream(hp):
        loss = _train_step(model, optimizer, noisy, clean, clip_norm)
    cur.wait_stream(hp)
    loss.record_stream(cur)
    return loss


def _train_step(model, optimizer, noisy, clean, clip_norm):
    from .functional import deferred_weight_grads
    _, wav = model(noisy)
    target = reshape_wav_to_mono(clean)
    est = pad_or_truncate_wav(reshape_wav_to_mono(wav), target)
    loss = SI_SNR_loss(est, target)
    with deferred_weight_grads(_defer_ok(model)):
        loss.backward()
    if clip_norm:
        torch.nn.utils.clip_grad_norm_(model.parameters(), clip_norm)
    optimizer.step()
    optimizer.zero_grad(set_to_none=True)
    return loss.detach()


def setup_distributed(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env. Returns
    (rank, world_size, local_rank, device)."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world)
        if device.type == "cuda":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, local, device


def wrap_ddp(model, device):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=4, gradient_as_bucket_view=True)
