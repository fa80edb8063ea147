"""CRN backward: per-tensor gradient error of the HIP path (per conv-math mode)
and of the fp32 oracle, against the fp64 oracle, on the golden CRN input."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "speech-enhancement_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import paramfill
from oracle import models as O
from sehip import functional as F, models as M

g = np.load(os.path.join(ROOT, "tests/golden/model_crn.npz"))
x = torch.from_numpy(g["x"])
r = None


def oracle(dtype):
    global r
    m = paramfill.fill_(O.CRN(320, 160, 320), seed=25).to(dtype).train()
    _, w = m(x.to(dtype))
    if r is None:
        r = torch.randn(w.shape, generator=torch.Generator().manual_seed(3))
    (w * r.to(dtype)).sum().backward()
    return {n: p.grad.double() for n, p in m.named_parameters() if p.grad is not None}


g64, g32 = oracle(torch.float64), oracle(torch.float32)
for mode in sys.argv[1:] or [F.get_conv_math(), "f32"]:
    F.set_conv_math(mode)
    m = paramfill.fill_(M.CRN(320, 160, 320), seed=25).cuda().train()
    _, w = m(x.cuda())
    (w * r.cuda()).sum().backward()
    print("mode", mode)
    for n, p in m.named_parameters():
        if n not in g64:
            continue
        d = g64[n].norm().item() + 1e-30
        e = (p.grad.double().cpu() - g64[n]).norm().item() / d
        e32 = (g32[n] - g64[n]).norm().item() / d
        print(f"  {n:50s} hip {e:.2e}  fp32-oracle {e32:.2e}", flush=True)
