"""Feasibility micro for batch-split overlap of ComplexBatchNorm2d (HBM-bound) with the
conv GEMMs (MFMA-bound): FRCRN encoder layer 1 at B = 64 (x [64, 128, 158, 404] ->
conv (5, 2) stride (2, 1) -> CBN + LeakyReLU). Variants, per-iteration ms:
  serial : conv(B) ; cbn(B)                      (today's order on one stream)
  halves : conv(B/2) ; conv(B/2) ; cbn(B/2) ; cbn(B/2)   (same stream: the split's own cost)
  overlap: conv(h1) ; conv(h2) on s0 while cbn(h1) runs on s1 after conv(h1) ; cbn(h2) on s0
(the halves' CBN uses per-half statistics: a timing stand-in for the moments / apply
passes of one half)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip.complex_nn import ComplexBatchNorm2d, ComplexConv2d  # noqa: E402
from sehip import functional as F  # noqa: E402

dev = torch.device("cuda")
conv = ComplexConv2d(128, 128, (5, 2), stride=(2, 1)).to(dev)
bn = ComplexBatchNorm2d(128).to(dev).train()
x = torch.randn(64, 128, 158, 404, device=dev) * 0.5
s0 = torch.cuda.current_stream(dev)
s1 = torch.cuda.Stream(dev)


def cbn(y):
    return bn.forward_act(y, F.ACT_LEAKY, 0.2)


def serial():
    cbn(conv(x))


def halves():
    a, b = conv(x[:32]), conv(x[32:])
    cbn(a); cbn(b)


def overlap():
    a = conv(x[:32])
    ev = torch.cuda.Event(); ev.record(s0)
    b = conv(x[32:])
    s1.wait_event(ev)
    with torch.cuda.stream(s1):
        cbn(a)
    a.record_stream(s1)
    cbn(b)
    s0.wait_stream(s1)


with torch.no_grad():
    for name, f in (("serial", serial), ("halves", halves), ("overlap", overlap)) * 2:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:8s} {e0.elapsed_time(e1) / 10:7.3f} ms", flush=True)
    yfull = torch.randn(64, 128, 77, 403, device=dev)
    for name, f in (("conv", lambda: conv(x)), ("cbn", lambda: cbn(yfull))):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:8s} {e0.elapsed_time(e1) / 10:7.3f} ms", flush=True)
