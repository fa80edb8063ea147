"""Kernel split of the fused CCBAM at the largest FRCRN skip (F=158)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402
from sehip.ccbam import CCBAM  # noqa: E402
dev = torch.device("cuda:0")
m = CCBAM(128).to(dev).train()
x = torch.randn(64, 128, 158, 403, device=dev, requires_grad=True)
g = torch.randn_like(x)
for _ in range(2):
    m(x).backward(g)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    m(x).backward(g)
    torch.cuda.synchronize()
for e in sorted(prof.key_averages(), key=lambda e: -e.self_device_time_total)[:25]:
    if e.self_device_time_total > 0:
        print(f"{e.self_device_time_total / 1e3:8.3f} ms {e.count:4d}  {e.key[:120]}")
