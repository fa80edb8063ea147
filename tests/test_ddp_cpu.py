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
