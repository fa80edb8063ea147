"""Few-dispatch microbenchmark of the HIP ops at the bench shapes (FRCRN,
B=64, 4 s @ 16 kHz) for rocprofv3 PMC passes: ConvSTFT fwd, ConviSTFT
fwd/bwd, and the enc1 / dec5 complex-conv GEMM passes."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip.conv_stft import ConvSTFT, ConviSTFT

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda")
x = torch.randn(64, 64000, device=dev) * 0.3
st, ist = ConvSTFT(320, 160, 640).to(dev), ConviSTFT(320, 160, 640).to(dev)
spec = st(x).detach().requires_grad_(True)
for name, f in [("stft_fwd", lambda: st(x)), ("istft_fwd", lambda: ist(spec)),
                ("istft_fwd+bwd", lambda: ist(spec).sum().backward())]:
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        f()
    torch.cuda.synchronize()
    print(f"{name:14s} {(time.perf_counter() - t0) / iters * 1e3:8.3f} ms", flush=True)
sys.argv = [sys.argv[0], "--iters", "1", "--layers", "enc1,dec5"]
exec(open(os.path.join(ROOT, "tools", "conv_micro.py")).read())
