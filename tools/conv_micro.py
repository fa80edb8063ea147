"""Microbenchmark of the complex-conv GEMM passes at FRCRN B=64 layer shapes
(for rocprofv3 PMC collection and A/B timing of kernel variants)."""
import argparse, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip import functional as F

LAYERS = {  # name: (transposed, cin, cout, input shape)
    "enc1": (False, 128, 128, (64, 128, 158, 404)),
    "dec5": (True, 256, 128, (64, 256, 158, 403)),
    "dec3": (True, 256, 128, (64, 256, 37, 403)),
    "enc4": (False, 128, 128, (64, 128, 17, 404)),
}
ap = argparse.ArgumentParser()
ap.add_argument("--layers", default="enc1,dec5")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--passes", default="fwd,data,weight")
ap.add_argument("--math", default="f32,bf16x3,bf16x6", help="conv math modes to time (se_conv2d_desc.math)")
args = ap.parse_args()
dev = torch.device("cuda")
for name in args.layers.split(","):
    tr, cin, cout, shape = LAYERS[name]
    x = torch.randn(shape, device=dev)
    wshape = (cin // 2, cout // 2, 5, 2) if tr else (cout // 2, cin // 2, 5, 2)
    wr = torch.randn(wshape, device=dev) * 0.05
    wi = torch.randn(wshape, device=dev) * 0.05
    d = F.conv_desc(shape, cout, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), tr, True)
    d.math = 0
    lib = F.N.lib()
    ho, wo = F.N.c_int(), F.N.c_int()
    lib.se_conv2d_out_shape(F.N.ctypes.byref(d), F.N.ctypes.byref(ho), F.N.ctypes.byref(wo))
    y = torch.randn(shape[0], cout, ho.value, wo.value, device=dev)
    dx = torch.empty_like(x)
    dwr, dwi = torch.empty_like(wr), torch.empty_like(wi)
    ws = torch.empty(lib.se_conv2d_workspace_size(F.N.ctypes.byref(d)), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    fl = F._conv_flops(d)
    calls = {
        "fwd": lambda: lib.se_conv2d_fwd(F.N.ctypes.byref(d), x.data_ptr(), wr.data_ptr(), wi.data_ptr(), None, None, y.data_ptr(), ws.data_ptr(), ws.numel(), st),
        "data": lambda: lib.se_conv2d_bwd_data(F.N.ctypes.byref(d), y.data_ptr(), wr.data_ptr(), wi.data_ptr(), dx.data_ptr(), ws.data_ptr(), ws.numel(), st),
        "weight": lambda: lib.se_conv2d_bwd_weight(F.N.ctypes.byref(d), x.data_ptr(), y.data_ptr(), dwr.data_ptr(), dwi.data_ptr(), None, None, ws.data_ptr(), ws.numel(), st),
    }
    outs = {"fwd": lambda: y, "data": lambda: dx, "weight": lambda: dwr}
    y0 = y.clone()
    for p in args.passes.split(","):
        f = calls[p]
        ref = None
        for mname in args.math.split(","):
            d.math = F._MATH_CODES[mname]
            if p == "fwd":
                y.copy_(y0)   # the data-grad pass reads y as dy
            assert f() == 0
            torch.cuda.synchronize()
            out = outs[p]().clone()
            err = "" if ref is None else f"  rel-L2 vs {args.math.split(',')[0]} {((out - ref).norm() / ref.norm()).item():.2e}"
            ref = out if ref is None else ref
            t0 = time.perf_counter()
            for _ in range(args.iters):
                f()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.iters
            print(f"{name:5s} {p:6s} {mname:6s} {dt*1e3:8.2f} ms  {fl/dt/1e12:7.1f} TF{err}", flush=True)
        if p == "fwd":
            y.copy_(y0)
