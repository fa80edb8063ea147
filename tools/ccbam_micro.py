"""CCBAM fwd+bwd at the six FRCRN B=64 skip shapes (128 ch x F x 403)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement_amd"))
import torch  # noqa: E402

from sehip.ccbam import CCBAM  # noqa: E402

dev = torch.device("cuda:0")
F_ROWS = [158, 77, 37, 17, 7, 2]
mods = [CCBAM(128).to(dev).train() for _ in F_ROWS]
xs = [torch.randn(64, 128, f, 403, device=dev, requires_grad=True) for f in F_ROWS]
gs = [torch.randn(64, 128, f, 403, device=dev) for f in F_ROWS]


def run(iters):
    for _ in range(iters):
        for m, x, g in zip(mods, xs, gs):
            m(x).backward(g)


run(2)
torch.cuda.synchronize()
t = time.perf_counter()
run(5)
torch.cuda.synchronize()
tot = (time.perf_counter() - t) / 5 * 1e3
for m, x, g in zip(mods, xs, gs):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        m(x).backward(g)
    torch.cuda.synchronize()
    print(f"  F={x.shape[2]:4d}  {(time.perf_counter() - t) / 5 * 1e3:7.2f} ms  "
          f"({x.numel() * 4 / 1e9:.2f} GB per pass)")
print(f"CCBAM fwd+bwd, all six skips: {tot:.2f} ms")
