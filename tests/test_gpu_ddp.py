"""DDP over the HIP ops on the one-GPU box: two ranks share cuda:0 and talk
gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's
scaling bench). Checks that the custom autograd Functions behave under
DistributedDataParallel: replicas end bit-identical and the gradients are the
mean of the per-shard gradients."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import paramfill

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank):
    noisy, clean = paramfill.structured_pair(2, 16000, seed=60 + rank)
    return torch.from_numpy(noisy), torch.from_numpy(clean)


def _worker(rank, world, port, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from sehip.models import FRCRN
    from sehip.losses import SI_SNR_loss
    from sehip.train import finish_grads, setup_distributed, wrap_ddp
    _, _, _, dev = setup_distributed(backend="gloo")
    model = paramfill.fill_(FRCRN(), seed=9).to(dev).train()
    ddp = wrap_ddp(model, dev, mode)
    noisy, clean = (t.to(dev) for t in _shard(rank))
    _, wav = ddp(noisy)
    SI_SNR_loss(wav, clean).backward()
    finish_grads(ddp)
    torch.cuda.synchronize()
    torch.save({n: p.grad.detach().cpu() for n, p in model.named_parameters()},
               os.path.join(out_dir, f"g{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("mode", ["flat", "ddp"])
def test_ddp_two_ranks_one_gpu(tmp_path, gpu_device, mode):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), mode), nprocs=world, join=True)
    g = [torch.load(tmp_path / f"g{r}.pt", weights_only=True) for r in range(world)]
    from sehip.models import FRCRN
    from sehip.losses import SI_SNR_loss
    per = []
    for r in range(world):
        m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
        noisy, clean = (t.cuda() for t in _shard(r))
        _, wav = m(noisy)
        SI_SNR_loss(wav, clean).backward()
        per.append({n: p.grad.detach().cpu() for n, p in m.named_parameters()})
    rels = []
    for n in g[0]:
        assert torch.equal(g[0][n], g[1][n]), n
        mean = (per[0][n] + per[1][n]) / 2
        rels.append(float((g[0][n] - mean).norm() / (mean.norm() + 1e-12)))
    rels.sort()
    assert rels[len(rels) // 2] < 1e-5 and rels[-1] < 1e-3, (rels[len(rels) // 2], rels[-1])


def _rccl_worker(rank, port, out_dir):
    """One rank over RCCL ("nccl" on ROCm): FlatDataParallel's broadcasts and its one
    flattened gradient all-reduce execute on RCCL (a world of one is the most this
    one-GPU box can host; RCCL refuses two ranks on one device)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from sehip.losses import SI_SNR_loss
    from sehip.models import FRCRN
    from sehip.train import FlatDataParallel, finish_grads, train_step, make_optimizer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    model = paramfill.fill_(FRCRN(), seed=9).to(dev).train()
    ddp = FlatDataParallel(model)
    noisy, clean = (t.to(dev) for t in _shard(0))
    _, wav = ddp(noisy)
    SI_SNR_loss(wav, clean).backward()
    finish_grads(ddp)
    torch.cuda.synchronize()
    torch.save({n: p.grad.detach().cpu() for n, p in model.named_parameters()}, os.path.join(out_dir, "g.pt"))
    # a full train step (forward, SI-SNR, backward, all-reduce, clip, AdamW) through the wrapper
    opt = make_optimizer(model)
    loss = train_step(ddp, opt, noisy, clean)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all()
    with open(os.path.join(out_dir, "rccl.txt"), "w") as f:
        f.write(str(torch.cuda.nccl.version()))
    dist.destroy_process_group()


def test_flat_ddp_over_rccl_world_one(tmp_path, gpu_device):
    port = _free_port()
    mp.spawn(_rccl_worker, args=(port, str(tmp_path)), nprocs=1, join=True)
    g = torch.load(tmp_path / "g.pt", weights_only=True)
    from sehip.models import FRCRN
    from sehip.losses import SI_SNR_loss
    m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
    noisy, clean = (t.cuda() for t in _shard(0))
    _, wav = m(noisy)
    SI_SNR_loss(wav, clean).backward()
    for n, p in m.named_parameters():   # the mean over one rank: the local gradient
        ref = p.grad.cpu()
        assert ((g[n] - ref).norm() / ref.norm().clamp_min(1e-30)).item() < 1e-5, n
    assert (tmp_path / "rccl.txt").read_text()
