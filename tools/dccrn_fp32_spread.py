"""How far independent fp32 evaluations of DCCRN-CL's training gradients land from fp64
(the anchor of tests/test_gpu_models.py::test_dccrn_train_grads_vs_fp64):
the fp32 CPU oracle at 1 / 4 / 8 threads and with 2^-22 relative input perturbations, each
as the median and max per-tensor rel-L2 against the unperturbed fp64 oracle, plus the fp64
oracle's own move under the same perturbations.  python tools/dccrn_fp32_spread.py"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch
from test_gpu_models import _dccrn_grads

g64 = _dccrn_grads("cpu", torch.float64)


def stats(g):
    e = [(g[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30) for n in g64]
    return np.median(e), max(e)


rows = []
for th in (1, 4, 8):
    torch.set_num_threads(th)
    rows.append((f"fp32 oracle, {th} threads", *stats(_dccrn_grads("cpu", torch.float32))))
torch.set_num_threads(8)
for i in range(3):
    rows.append((f"fp32 oracle, input x (1 + 2^-22 N(0,1)), seed {1234 + i}",
                 *stats(_dccrn_grads("cpu", torch.float32, perturb=2.0 ** -22, seed=1234 + i))))
for i in range(3):
    rows.append((f"fp64 oracle, input x (1 + 2^-22 N(0,1)), seed {1234 + i}",
                 *stats(_dccrn_grads("cpu", torch.float64, perturb=2.0 ** -22, seed=1234 + i))))
print(f"{'evaluation':62s} {'median':>9s} {'max':>9s}   (per-tensor rel-L2 vs unperturbed fp64, {len(g64)} tensors)")
for name, med, mx in rows:
    print(f"{name:62s} {med:9.2e} {mx:9.2e}")
