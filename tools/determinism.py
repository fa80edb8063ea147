"""Run-to-run determinism of the FRCRN train-step gradients on the HIP path
(same weights, same inputs, twice in one process): every kernel is expected
to be bitwise deterministic (no atomics on the data path)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import paramfill
from sehip import functional as F
from sehip.models import FRCRN
from sehip.losses import SI_SNR_loss

for math in sys.argv[1:] or ["f32", "bf16x3"]:
    F.set_conv_math(math)
    grads = []
    for rep in range(3):
        m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
        noisy, clean = (torch.from_numpy(t).cuda() for t in paramfill.structured_pair(2, 16000, seed=60))
        _, wav = m(noisy)
        SI_SNR_loss(wav, clean).backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    bad = [n for n in grads[0] if not (torch.equal(grads[0][n], grads[1][n]) and torch.equal(grads[0][n], grads[2][n]))]
    worst = max(((grads[0][n] - grads[1][n]).norm() / (grads[0][n].norm() + 1e-30)).item() for n in grads[0])
    print(f"{math}: {len(bad)} of {len(grads[0])} grads differ between runs; worst rel {worst:.2e}; first: {bad[:6]}", flush=True)
