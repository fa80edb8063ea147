"""ComplexBatchNorm2d (+ LeakyReLU) forward / backward alone at the FRCRN bench
shapes (B = 64, 128 channels; the encoder's forked outputs go through
se_cbn_bwd2, the decoder's through se_cbn_bwd), timed with HIP events: the HBM
rate of each pass by the bytes it must move (fwd: x read twice + y written;
bwd: x, gy (+ gy2) read twice + dx written). Run it under rocprofv3
--kernel-trace --stats to split the passes per kernel.
  python tools/cbn_micro.py [--iters N] [--only enc|dec]"""
import argparse, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip.complex_nn import ComplexBatchNorm2d
from sehip import functional as F

# (F, T) of the 128-channel CBN inputs in FRCRN at 4 s (oracle FRCRN, forward hooks)
ENC = [(158, 403), (77, 403), (37, 403), (17, 403), (7, 403), (2, 403)]
DEC = [(7, 404), (17, 404), (37, 404), (77, 404), (157, 404)]

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--only", default="")
ap.add_argument("--B", type=int, default=64)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
tot = {"fwd": [0.0, 0.0], "bwd": [0.0, 0.0]}
for tag, shapes, fork in (("enc", ENC, True), ("dec", DEC, False)):
    if a.only and a.only != tag:
        continue
    for (f, t) in shapes:
        bn = ComplexBatchNorm2d(128).to(dev).train()
        x = torch.randn(a.B, 128, f, t, device=dev).requires_grad_(True)
        gys = [torch.randn(a.B, 128, f, t, device=dev) for _ in range(2 if fork else 1)]
        nb = x.numel() * 4
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf = tb = 0.0
        for it in range(a.iters + 1):
            ev[0].record()
            out = bn.forward_act(x, F.ACT_LEAKY, 0.01, fork)
            ev[1].record()
            outs = out if fork else (out,)
            torch.autograd.backward(outs, gys)
            ev[2].record()
            torch.cuda.synchronize()
            if it:
                tf += ev[0].elapsed_time(ev[1]) / a.iters
                tb += ev[1].elapsed_time(ev[2]) / a.iters
            x.grad = None
        fb, bb = 3 * nb, (2 * (1 + len(gys)) + 1) * nb
        tot["fwd"][0] += tf; tot["fwd"][1] += fb
        tot["bwd"][0] += tb; tot["bwd"][1] += bb
        print(f"{tag} F={f:3d} T={t} {nb / 1e9:6.3f} GB/tensor  fwd {tf:7.3f} ms {fb / tf / 1e9:6.2f} TB/s"
              f"  bwd {tb:7.3f} ms {bb / tb / 1e9:6.2f} TB/s", flush=True)
for k, (ms, by) in tot.items():
    if ms:
        print(f"total {k}: {ms:7.3f} ms  {by / ms / 1e9:6.2f} TB/s")
