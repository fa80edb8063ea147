"""Each CCBAM full-tensor pass (csrc/ccbam.hip) alone at the FRCRN B = 64 skip shapes:
per-launch time over a burst of back-to-back launches and GB/s of the pass's own
algorithmic bytes (each full-size operand read once, each output written once)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import torch  # noqa: E402

from sehip import _native as N  # noqa: E402
from sehip import functional as F  # noqa: E402

dev = torch.device("cuda")
lib = N.lib()
B, C = 64, 128


def burst(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for Fr in [int(a) for a in (sys.argv[1:] or ["158", "77", "17", "2"])]:
    HW = Fr * 403
    x = torch.randn(B, C, HW, device=dev)
    g = torch.randn(B, C, HW, device=dev)
    out = torch.empty_like(x)
    dx = torch.empty_like(x)
    mean, mx = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
    am = torch.empty(B, C, device=dev, dtype=torch.int32)
    ca = torch.rand(B, C, device=dev)
    P = torch.empty(B, 4, HW, device=dev)
    idx = torch.zeros(B, 2, HW, device=dev, dtype=torch.int16)
    sa = torch.rand(B, 2, HW, device=dev)
    dz = torch.empty(B, 2, HW, device=dev)
    dP = torch.randn(B, 4, HW, device=dev)
    dca = torch.empty(B, C, device=dev)
    ws = F._workspace(lib.se_ccbam_workspace_size(B, C, HW), dev)
    oa = torch.empty(1, device=dev)
    st = N.stream_of(x)
    T = x.numel() * 4
    runs = [
        ("channel_pool", 1, lambda: lib.se_ccbam_channel_pool(x.data_ptr(), mean.data_ptr(), mx.data_ptr(),
                                                               am.data_ptr(), B, C, HW, st)),
        ("spatial_pool", 1, lambda: lib.se_ccbam_spatial_pool(x.data_ptr(), ca.data_ptr(), P.data_ptr(),
                                                               idx.data_ptr(), B, C, HW, st)),
        ("apply", 2, lambda: lib.se_ccbam_apply(x.data_ptr(), ca.data_ptr(), sa.data_ptr(), out.data_ptr(), B, C, HW,
                                                oa.data_ptr(), st)),
        ("bwd_sa_sigmoid", 1, lambda: lib.se_ccbam_bwd_sa_sigmoid(g.data_ptr(), sa.data_ptr(), dz.data_ptr(), B, C, HW,
                                                                  st)),
        ("bwd_dca", 2, lambda: lib.se_ccbam_bwd_dca(g.data_ptr(), x.data_ptr(), dP.data_ptr(), idx.data_ptr(),
                                                    dca.data_ptr(), B, C, HW, ws.data_ptr(), ws.numel(), st)),
        ("bwd_dx", 2, lambda: lib.se_ccbam_bwd_dx(g.data_ptr(), dP.data_ptr(), idx.data_ptr(), ca.data_ptr(),
                                                  mean.data_ptr(), mx.data_ptr(), am.data_ptr(), dx.data_ptr(), B, C,
                                                  HW, st)),
    ]
    tot = 0.0
    for name, passes, fn in runs:
        ms = burst(fn)
        tot += ms
        print(f"F={Fr:4d} {name:15s} {ms * 1e3:8.1f} us  {passes * T / ms / 1e6:8.1f} GB/s ({passes} passes of "
              f"{T / 1e9:.2f} GB)", flush=True)
    print(f"F={Fr:4d} all six passes {tot * 1e3:.1f} us", flush=True)
    del x, g, out, dx, P, idx, sa, dz, dP
    torch.cuda.empty_cache()
