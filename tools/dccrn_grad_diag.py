"""DCCRN-CL training-gradient error per parameter tensor against an fp64 CPU run of
the oracle, for several sehip configurations (which stage carries the error).
Usage (GPU box): python tools/dccrn_grad_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "speech-enhancement_amd"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
from test_gpu_models import _dccrn_grads   # noqa: E402


def main():
    from sehip import functional as F
    g64 = _dccrn_grads("cpu", torch.float64)
    g32 = _dccrn_grads("cpu", torch.float32)
    runs = {"oracle-fp32-cpu": g32}
    for name, math, lstm in (("default", "f16x3", "hip"), ("conv-f32", "f32", "hip"),
                             ("lstm-torch", "f16x3", "torch"), ("all-f32", "f32", "torch")):
        os.environ["SEHIP_LSTM_GEMM"] = lstm
        F.set_conv_math(math)
        runs[name] = _dccrn_grads("cuda", torch.float32, sehip=True)
    F.set_conv_math("f16x3")
    os.environ["SEHIP_LSTM_GEMM"] = "hip"
    names = list(g64)
    err = {k: np.array([((g[n] - g64[n]).norm() / (g64[n].norm() + 1e-30)).item() for n in names])
           for k, g in runs.items()}
    print("median per-tensor rel-L2 vs fp64: " + "  ".join(f"{k} {np.median(v):.2e}" for k, v in err.items()))
    order = np.argsort(-err["default"])
    print("worst tensors (default):")
    for i in order[:40]:
        print(f"  {names[i]:60s} " + " ".join(f"{k}={err[k][i]:.1e}" for k in err))


if __name__ == "__main__":
    main()
