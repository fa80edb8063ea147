"""How well-conditioned are DCUNet's training gradients under its default 'bounded_tanh'
mask (/root/reference/models/_1903_03107_dcunet.py:158-184: phase = n_ph + m_ph / m_mag)?
CPU only (the oracle, oracle/models.py): per-tensor rel-L2 of fp32 evaluations and of
fp64 evaluations on 2^-22-perturbed inputs against the unperturbed fp64 gradient, for
DCUNet-16 and DCUNet-20 at random init (paramfill), on the structured pair of the
gradient gates. Prints one line per evaluation (median / max over tensors).

  python tools/dcunet_tanh_spread.py > profiles/r6_dcunet_tanh_spread.log
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import paramfill  # noqa: E402
from oracle import models as O, train as OT  # noqa: E402


def grads(cfg, dtype, mask, perturb=0.0, seed=1234, threads=None):
    if threads:
        torch.set_num_threads(threads)
    noisy, clean = paramfill.structured_pair(1, 32000, seed=42)
    m = paramfill.fill_(O.DCUNet(cfg, 512, 128, 512), seed=75).to(dtype).train()
    if mask == "bounded_sigmoid":
        m._mask = lambda h, noisy: noisy * torch.sigmoid(h)
    x = torch.from_numpy(noisy).to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=torch.float64)).to(dtype)
    c = torch.from_numpy(clean).to(dtype)
    _, w = m(x)
    OT.si_snr_loss(OT.pad_or_truncate_wav(w, c), c).backward()
    return {n: p.grad.detach().double() for n, p in m.named_parameters()}


def main():
    print("# DCUNet training gradients at random init: per-tensor rel-L2 vs the unperturbed fp64 gradient")
    print(f"# torch {torch.__version__}, {torch.get_num_threads()} threads")
    for cfg in ("dcunet16", "dcunet20"):
        for mask in ("bounded_tanh", "bounded_sigmoid"):
            g64 = grads(cfg, torch.float64, mask)
            rows = [("fp32", grads(cfg, torch.float32, mask))]
            rows += [(f"fp64, input x (1 + 2^-22 N(0,1)) seed {1234 + i}",
                      grads(cfg, torch.float64, mask, perturb=2.0 ** -22, seed=1234 + i)) for i in range(2)]
            rows += [(f"fp32, input x (1 + 2^-22 N(0,1)) seed {1234 + i}",
                      grads(cfg, torch.float32, mask, perturb=2.0 ** -22, seed=1234 + i)) for i in range(2)]
            for name, g in rows:
                rel = [(g[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30) for n in g64]
                print(f"{cfg:9s} {mask:16s} {name:45s} median {np.median(rel):.2e}  max {max(rel):.2e}", flush=True)


if __name__ == "__main__":
    main()
