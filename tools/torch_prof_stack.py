"""Which source lines launch the copy / cat / pad / add kernels in one FRCRN
train step (torch.profiler with stacks). Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from sehip.data import synthetic_pairs  # noqa: E402
from sehip.models import FRCRN  # noqa: E402
from sehip.train import make_optimizer, train_step  # noqa: E402

dev = torch.device("cuda:0")
model = FRCRN().to(dev).train()
opt = make_optimizer(model)
noisy, clean = synthetic_pairs(64, 64000, device=dev)
for _ in range(2):
    train_step(model, opt, noisy, clean)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    train_step(model, opt, noisy, clean)
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_stack_n=6)
want = ("aten::copy_", "aten::cat", "aten::constant_pad_nd", "aten::add_", "aten::add", "aten::fill_",
        "aten::contiguous", "aten::clone", "aten::mul", "aten::sum", "aten::zero_")
rows = [e for e in ka if e.key in want and e.device_time_total > 200]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:40]:
    st = [s for s in e.stack if "sehip" in s or "torch/autograd" in s or "torch/nn" in s][:3]
    print(f"{e.device_time_total / 1e3:8.2f} ms {e.count:4d}  {e.key:22s} {' | '.join(st)[:230]}")
