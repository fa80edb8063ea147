"""Data-parallel path on the CPU (gloo, world_size 2), SURVEY.md §8(e).

The launcher (sehip.train.setup_distributed / wrap_ddp / train_step) is run
with the oracle FRCRN on the CPU: after one DDP step every rank must hold
the average of the per-shard gradients (computed here single-process), the
replicas must stay bit-identical, and ComplexBatchNorm keeps per-rank
statistics (DDP semantics; the reference has no SyncBN).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import paramfill

pytestmark = pytest.mark.timeout(600) if hasattr(pytest.mark, "timeout") else []


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank):
    noisy, clean = paramfill.structured_pair(2, 8000, seed=40 + rank)
    return torch.from_numpy(noisy), torch.from_numpy(clean)


def _worker(rank, world, port, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from oracle import models as O
    from sehip.train import FlatDataParallel, finish_grads, setup_distributed, wrap_ddp, train_step
    r, w, _, dev = setup_distributed(backend="gloo")
    assert (r, w, dev.type) == (rank, world, "cpu")
    model = paramfill.fill_(O.FRCRN(), seed=7).train()
    ddp = wrap_ddp(model, dev, mode)
    assert isinstance(ddp, FlatDataParallel if mode == "flat" else torch.nn.parallel.DistributedDataParallel)
    noisy, clean = _shard(rank)
    # grads of one step without the optimiser update (clip disabled, lr 0)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.0)
    _, wav = ddp(noisy)
    from sehip.losses import SI_SNR_loss
    SI_SNR_loss(wav, clean).backward()
    finish_grads(ddp)
    grads = {n: p.grad.clone() for n, p in model.named_parameters()}
    torch.save({"grads": grads, "RMr": model.encoder.layers[0].norm.RMr.clone()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    opt.zero_grad()
    # and a full packaged step runs under DDP
    loss = train_step(ddp, torch.optim.AdamW(ddp.parameters(), lr=1e-3), noisy, clean)
    assert torch.isfinite(loss)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("mode", ["flat", "ddp"])
def test_ddp_gloo_world2_grad_average(tmp_path, mode):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), mode), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # replicas agree exactly after the all-reduce
    for n in res[0]["grads"]:
        assert torch.equal(res[0]["grads"][n], res[1]["grads"][n]), n
    # and equal the mean of the single-process per-shard gradients
    from oracle import models as O
    from sehip.losses import SI_SNR_loss
    torch.set_num_threads(2)          # same intra-op reduction order as the workers
    per = []
    for r in range(world):
        m = paramfill.fill_(O.FRCRN(), seed=7).train()
        noisy, clean = _shard(r)
        _, wav = m(noisy)
        SI_SNR_loss(wav, clean).backward()
        per.append({n: p.grad for n, p in m.named_parameters()})
    worst = 0.0
    for n in per[0]:
        mean = (per[0][n] + per[1][n]) / world
        d = (res[0]["grads"][n] - mean).norm() / (mean.norm() + 1e-12)
        worst = max(worst, float(d))
    assert worst < 1e-4, worst
    # per-rank BN statistics (no SyncBN): each rank updated its running mean from its own shard
    assert not torch.equal(res[0]["RMr"], res[1]["RMr"])


def _unused_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from sehip.train import FlatDataParallel, setup_distributed
    setup_distributed(backend="gloo")
    torch.manual_seed(0)
    net = torch.nn.ModuleDict({"a": torch.nn.Linear(4, 3), "b": torch.nn.Linear(4, 5), "c": torch.nn.Linear(4, 2)})
    ddp = FlatDataParallel(net)
    x = torch.full((2, 4), float(rank + 1))
    # rank 0 leaves "b" unused, rank 1 leaves "c" unused: per-rank grad sets differ
    out = net["a"](x).sum() + (net["c"](x).sum() if rank == 0 else net["b"](x).sum())
    out.backward()
    ddp.allreduce_grads()
    torch.save({n: p.grad.clone() for n, p in net.named_parameters()}, os.path.join(out_dir, f"u{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_flat_dp_unused_parameters_differ_by_rank(tmp_path):
    """FlatDataParallel flattens every trainable parameter (zeros for a missing
    gradient), so ranks whose unused-parameter sets differ still all-reduce
    identically laid-out buffers: every rank ends with the DDP average."""
    world, port = 2, _free_port()
    mp.spawn(_unused_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    g = [torch.load(tmp_path / f"u{r}.pt", weights_only=True) for r in range(world)]
    for n in g[0]:
        assert torch.equal(g[0][n], g[1][n]), n
    # d sum(W x) / dW = sum over the 2 rows of x = 2 (rank + 1); "b" got a gradient only on
    # rank 1 (4), averaged with rank 0's zeros; "c" only on rank 0 (2); "a" on both (2, 4)
    assert torch.allclose(g[0]["b.weight"], torch.full((5, 4), 4.0 / 2))
    assert torch.allclose(g[0]["c.weight"], torch.full((2, 4), 2.0 / 2))
    assert torch.allclose(g[0]["a.weight"], torch.full((3, 4), (2.0 + 4.0) / 2))
