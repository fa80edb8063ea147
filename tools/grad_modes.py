"""Gradient error of the FRCRN train step per conv-math mode (per pass)
against the fp64 oracle, on the golden train-step pair: which passes can run
split-bf16 and keep the per-tensor gate of tests/test_gpu_models.py."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "speech-enhancement_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import paramfill
from oracle import models as O, train as OT
from sehip import functional as F, models as M
from sehip.losses import SI_SNR_loss, pad_or_truncate_wav
g = np.load(os.path.join(ROOT, "tests/golden/train_step_frcrn.npz"))
noisy, clean = torch.from_numpy(g["noisy"]), torch.from_numpy(g["clean"])


def oracle_grads(dtype, perturb=0.0):
    x = noisy.to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(1234)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=dtype))
    m = paramfill.fill_(O.FRCRN(), seed=30).to(dtype).train()
    _, w = m(x[:, None])
    OT.si_snr_loss(OT.pad_or_truncate_wav(w, clean.to(dtype)), clean.to(dtype)).backward()
    return {n: p.grad.double() for n, p in m.named_parameters()}


g64, g32, g32p = oracle_grads(torch.float64), oracle_grads(torch.float32), oracle_grads(torch.float32, 2.0 ** -22)
modes = sys.argv[1:] or ["f32", "bf16x3", "fwd=bf16x3,data=f32,weight=f32", "fwd=f32,data=bf16x3,weight=f32",
                         "fwd=f32,data=f32,weight=bf16x3", "fwd=bf16x3,data=f32,weight=bf16x3"]
for mode in modes:
    F.set_conv_math(mode)
    m = paramfill.fill_(M.FRCRN(), seed=30).cuda().train()
    _, w = m(noisy.cuda()[:, None])
    wrel = ((w.detach().cpu().double() - torch.from_numpy(g["wav"]).double()).norm() / np.linalg.norm(g["wav"])).item()
    SI_SNR_loss(pad_or_truncate_wav(w, clean.cuda()), clean.cuda()).backward()
    errs = []
    for n, p in m.named_parameters():
        d = g64[n].norm().item() + 1e-30
        e = (p.grad.double().cpu() - g64[n]).norm().item() / d
        lim = max(3 * (g32[n] - g64[n]).norm().item() / d, 3 * (g32p[n] - g32[n]).norm().item() / d, 1e-3)
        errs.append((e / lim, e, n))
    errs.sort(reverse=True)
    med = np.median([e[1] for e in errs])
    med32 = np.median([(g32[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30) for n in g64])
    print(f"{mode:40s} wav {wrel:.1e} grads: worst err/limit {errs[0][0]:.2f} ({errs[0][2]}), "
          f"{sum(e[0] > 1 for e in errs)} over; median {med:.1e} (fp32 oracle {med32:.1e})", flush=True)
