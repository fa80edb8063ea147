"""Op-level attribution of one FRCRN B=64 train step (torch.profiler):
aten ops sorted by device time, with input shapes. Diagnostic only."""
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
ka = prof.key_averages(group_by_input_shape=True)
rows = sorted(ka, key=lambda e: -e.self_device_time_total)
print(f"{'self dev ms':>11} {'calls':>5}  op  [shapes]")
for e in rows[:int(sys.argv[1]) if len(sys.argv) > 1 else 60]:
    if e.self_device_time_total <= 0:
        continue
    print(f"{e.self_device_time_total / 1e3:11.2f} {e.count:5d}  {e.key}  {str(e.input_shapes)[:150]}")
