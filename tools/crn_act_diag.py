"""CRN backward: gradient of every block output (decoder / encoder layers, LSTM) on
the HIP path vs the CPU oracle (fp32), to locate where the gradients depart."""
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


def run(m, dev):
    outs = {}
    def mk(name):
        def hook(mod, i, o):
            t = o[0] if isinstance(o, tuple) else o
            t.retain_grad()
            outs[name] = (t, i[0])
            if i[0].requires_grad:
                i[0].retain_grad()
        return hook
    for n, mod in m.named_modules():
        if n.startswith(("encoder.layers.", "decoder.layers.")) and n.count(".") == 2 or n.endswith((".conv", ".conv_transposed", ".norm", ".act")):
            mod.register_forward_hook(mk(n))
    _, w = m(x.to(dev))
    r = torch.randn(w.shape, generator=torch.Generator().manual_seed(3)).to(dev)
    (w * r).sum().backward()
    return {k: (o.grad.detach().cpu() if o.grad is not None else None, o.detach().cpu(),
                i.grad.detach().cpu() if i.grad is not None else None) for k, (o, i) in outs.items()}


F.set_conv_math(sys.argv[1] if len(sys.argv) > 1 else "f32")
mo = paramfill.fill_(O.CRN(320, 160, 320), seed=25).train()
mh = paramfill.fill_(M.CRN(320, 160, 320), seed=25).cuda().train()
ro, rh = run(mo, "cpu"), run(mh, "cuda")
def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30)) if a is not None and b is not None else float("nan")
for k in ro:
    if k in rh:
        print(f"{k:40s} out {rel(rh[k][1], ro[k][1]):.2e}  d_out {rel(rh[k][0], ro[k][0]):.2e}  d_in {rel(rh[k][2], ro[k][2]):.2e}", flush=True)
