"""Per-step wall time of the bench's FRCRN training step (synchronised after every step)
for a given number of seconds: shows when in a process's life GPU stalls fall.

  python tools/step_timeline.py [seconds, default 30]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
t_start = time.time()
import torch  # noqa: E402

from sehip.data import synthetic_pairs  # noqa: E402
from sehip.models import FRCRN  # noqa: E402
from sehip.train import make_optimizer, train_step  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda")
torch.manual_seed(2023)
model = FRCRN().to(dev).train()
opt = make_optimizer(model)
batches = [synthetic_pairs(64, 64000, seed=2023 + i, device=dev) for i in range(2)]
torch.cuda.synchronize()
print(f"# setup {time.time() - t_start:.2f} s after process start", flush=True)
t0 = time.time()
i = 0
while time.time() - t0 < secs:
    s = time.perf_counter()
    for _ in range(k):
        train_step(model, opt, *batches[i % 2])
        i += 1
    torch.cuda.synchronize()
    print(f"{time.time() - t_start:8.3f} s  step {i - k:4d}  {1e3 * (time.perf_counter() - s) / k:8.2f} ms", flush=True)
