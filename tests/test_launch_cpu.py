"""bench.py's multi-rank launch, on the CPU.

`python bench.py --gpus N` without torchrun spawns the N ranks itself
(sehip.train.spawn_ranks) and must never run fewer ranks than asked; under
torchrun `--gpus` must equal WORLD_SIZE. The reference's own DDP path
(/root/reference/trainer.py:53-55, train.py:53) never initialised a process
group; this is the launcher that replaces it.
"""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_more_gpus_than_visible():
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "only 0 GPU(s) visible" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def _rank_target(out_dir):
    from sehip.train import setup_distributed
    rank, world, local, dev = setup_distributed(backend="gloo")
    t = torch.tensor([float(rank + 1)])
    torch.distributed.all_reduce(t)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{rank} {world} {local} {os.environ['MASTER_ADDR']} {t.item()}")
    torch.distributed.destroy_process_group()


def _failing_target(out_dir):
    if int(os.environ["RANK"]) == 1:
        raise RuntimeError("rank 1 fails")


@pytest.mark.timeout(300)
def test_spawn_ranks_gloo(tmp_path):
    from sehip.train import spawn_ranks
    spawn_ranks(3, _rank_target, (str(tmp_path),))
    rows = sorted((tmp_path / f"r{r}.txt").read_text().split() for r in range(3))
    assert [r[:4] for r in rows] == [[str(r), "3", str(r), "127.0.0.1"] for r in range(3)]
    assert all(float(r[4]) == 6.0 for r in rows)


@pytest.mark.timeout(300)
def test_spawn_ranks_propagates_failure(tmp_path):
    from sehip.train import spawn_ranks
    with pytest.raises(Exception, match="rank 1 fails"):
        spawn_ranks(2, _failing_target, (str(tmp_path),))
