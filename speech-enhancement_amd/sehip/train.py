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

from . import optim as _optim
from .losses import si_snr_loss_aligned

ADAMW = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)   # hparams/*.py
CLIP_NORM = 0.5                                                           # hyperparams.py:10


def make_optimizer(model, **overrides):
    """AdamW with the reference's hyper-parameters: sehip.optim.AdamW (one HIP
    launch per step and storage type) for contiguous CUDA parameters (fp32, or a
    bf16 / fp16 model's), torch.optim.AdamW otherwise (CPU)."""
    kw = dict(ADAMW)
    kw.update(overrides)
    params = list(model.parameters())
    if params and all(p.is_cuda and p.dtype in _optim.N.DTYPES and p.is_contiguous() for p in params):
        return _optim.AdamW(params, **kw)
    return torch.optim.AdamW(params, **kw)


def _clip(model, clip_norm):
    """clip_grad_norm_(model.parameters(), clip_norm) (trainer.py:216-218): the
    HIP slot kernels for CUDA gradients of one storage type (fp32 / bf16 / fp16)."""
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    if grads and all(g.is_cuda and g.dtype == grads[0].dtype and g.dtype in _optim.N.DTYPES and g.is_contiguous()
                     for g in grads):
        return _optim.clip_grad_norm_(model.parameters(), clip_norm)
    return torch.nn.utils.clip_grad_norm_(model.parameters(), clip_norm)


def _defer_ok(model) -> bool:
    """Deferred weight-grads (functional.deferred_weight_grads) need every .grad
    None on entry and no gradient hooks during backward: not under hook-based DDP
    (FlatDataParallel reduces after backward and is fine), and only on the GPU."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    if isinstance(model, DDP):
        return False
    p = next(model.parameters(), None)
    return p is not None and p.is_cuda and all(q.grad is None for q in model.parameters()) \
        and os.environ.get("SEHIP_OVERLAP", "1") != "0"


_ONES: dict = {}


def _ones_like(t):
    key = (t.device, t.dtype, tuple(t.shape))
    o = _ONES.get(key)
    if o is None:
        o = _ONES[key] = torch.ones_like(t)
    return o


_INFLIGHT: list = []


def _throttle(dev):
    """Host flow control: at most SEHIP_MAX_INFLIGHT (default 2) steps queued on the GPU.
    A host far ahead of the GPU keeps every queued step's freed temporaries pinned (their
    uses on the side streams are recorded), the caching allocator grows past the step's
    working set, and at the HBM limit it frees its cache and allocates again: stalls of
    seconds when the driver is still clearing the previous process's memory
    (profiles/r6_host_runahead.log)."""
    depth = int(os.environ.get("SEHIP_MAX_INFLIGHT", "2"))
    if depth <= 0 or dev.type != "cuda":
        return
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    _INFLIGHT.append(ev)
    while len(_INFLIGHT) > depth:
        _INFLIGHT.pop(0).synchronize()


def train_step(model, optimizer, noisy, clean, clip_norm=CLIP_NORM):
    """One optimisation step; returns the (device) loss, no host sync (beyond keeping at
    most SEHIP_MAX_INFLIGHT steps queued, _throttle)."""
    from . import functional as F
    from .functional import deferred_weight_grads
    _, wav = model(noisy)
    loss = si_snr_loss_aligned(wav, clean)     # mono reshape + pad / truncate + SI-SNR
    with deferred_weight_grads(_defer_ok(model)):
        # the backward's seed dL/dL = 1 from a cached tensor (loss.backward() would fill a new one)
        torch.autograd.backward(loss, _ones_like(loss))
    finish_grads(model)
    if clip_norm:
        _clip(model, clip_norm)
    optimizer.step()
    optimizer.zero_grad(set_to_none=True)
    F.lstm_wide_poll()      # a wide-LSTM barrier timeout raises here, not as a NaN loss later
    _throttle(noisy.device)
    return loss.detach()


def setup_distributed(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env (or spawn_ranks'). Returns
    (rank, world_size, local_rank, device). With the GPU backend every local rank
    needs its own device: a rank whose LOCAL_RANK has no GPU raises instead of
    sharing another rank's."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # gloo rehearsals (tests, tools/gpu_ddp_rehearsal.sh) may put several ranks on one GPU
    shared_ok = (backend or os.environ.get("SEHIP_DIST_BACKEND")) == "gloo"
    if torch.cuda.is_available() and not shared_ok and local >= torch.cuda.device_count():
        raise RuntimeError(f"sehip: LOCAL_RANK {local} but only {torch.cuda.device_count()} visible GPU(s)")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        # SEHIP_DIST_BACKEND: override (e.g. gloo to rehearse ranks sharing one GPU)
        backend = backend or os.environ.get("SEHIP_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world)
        if device.type == "cuda":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, local, device


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, world, port, target, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      SEHIP_SPAWNED="1")
    target(*args)


def spawn_ranks(nprocs: int, target, args=(), port: int | None = None) -> None:
    """One fresh process per rank (torch.multiprocessing "spawn": a new
    interpreter each, so nothing the parent holds is inherited), with torchrun's
    environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT) set before ``target(*args)`` runs; ``setup_distributed`` in the
    target then binds cuda:LOCAL_RANK and joins the process group. The caller
    must not have initialised the GPU (device_count() does not). Raises if any
    rank fails (torch.multiprocessing.ProcessRaisedException / ProcessExitedException)."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_entry, args=(nprocs, port or free_port(), target, tuple(args)), nprocs=nprocs,
                       join=True, start_method="spawn")


class FlatDataParallel(torch.nn.Module):
    """Data parallelism with ONE gradient all-reduce after backward (RCCL over xGMI).

    Same semantics as DistributedDataParallel's defaults: parameters and buffers
    broadcast from rank 0 at construction, buffers (the CBN running statistics)
    broadcast from rank 0 at every forward, gradients averaged over ranks. The
    difference is where the reduction happens: DDP hooks every parameter's
    gradient and all-reduces 4-MB buckets during backward, which rules out the
    side streams of this path (the deferred weight-grads and the CCBAM gates: a
    hook would read a gradient its side-stream kernel has not written yet). The
    whole FRCRN gradient is 7.7 MB, a ~0.2 ms ring all-reduce against a ~120 ms
    step, so nothing is lost by reducing it once at the end, flattened, after the
    side streams have joined (train_step -> finish_grads)."""

    def __init__(self, module, process_group=None):
        super().__init__()
        import torch.distributed as dist
        self.module = module
        self.process_group = process_group
        self.world = dist.get_world_size(process_group)
        self._broadcast(list(module.parameters()) + list(module.buffers()))

    def _broadcast(self, tensors):
        """Rank 0's values, one coalesced broadcast per dtype (as DDP's buffer sync)."""
        import torch.distributed as dist
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        by_dtype: dict = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        with torch.no_grad():
            for ts in by_dtype.values():
                flat = _flatten_dense_tensors([t.detach() for t in ts])
                dist.broadcast(flat, 0, group=self.process_group)
                for t, v in zip(ts, _unflatten_dense_tensors(flat, ts)):
                    t.copy_(v)

    def forward(self, *args, **kwargs):
        self._broadcast(list(self.module.buffers()))
        return self.module(*args, **kwargs)

    def allreduce_grads(self):
        """Every trainable parameter takes part, in parameter order, so each rank
        contributes an identically laid-out buffer even if a parameter went
        unused on some rank (its gradient enters as zeros and, as under DDP,
        every rank then holds the averaged gradient)."""
        import torch.distributed as dist
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        params = [p for p in self.module.parameters() if p.requires_grad]
        if not params:
            return
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        grads = [p.grad for p in params]
        flat = _flatten_dense_tensors(grads)
        dist.all_reduce(flat, group=self.process_group)
        flat.div_(self.world)
        for g, r in zip(grads, _unflatten_dense_tensors(flat, grads)):
            g.copy_(r)


def finish_grads(model):
    """After backward: FlatDataParallel's gradient all-reduce (a no-op otherwise)."""
    if isinstance(model, FlatDataParallel):
        model.allreduce_grads()


def wrap_ddp(model, device, mode: str | None = None):
    """Data-parallel wrapper for world > 1 (identity otherwise). mode (or SEHIP_DP):
    "flat" (default) = FlatDataParallel, one all-reduce after backward, side streams
    kept; "ddp" = torch DistributedDataParallel (4-MB buckets during backward, side
    streams off)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    mode = mode or os.environ.get("SEHIP_DP", "flat")
    if mode == "flat":
        return FlatDataParallel(model)
    from torch.nn.parallel import DistributedDataParallel as DDP
    from . import functional as F
    F.DDP_HOOKS[0] = True   # gradient hooks during backward: no side streams (frcrn._overlap_ok)
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=4, gradient_as_bucket_view=True)
