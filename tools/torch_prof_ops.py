"""Device time of selected aten ops by input shape in one FRCRN train step."""
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
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    train_step(model, opt, noisy, clean)
    torch.cuda.synchronize()
want = sys.argv[1].split(",")
rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in want]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:40]:
    print(f"{e.device_time_total / 1e3:8.2f} ms {e.count:4d}  {e.key:24s} {str(e.input_shapes)[:160]}")
