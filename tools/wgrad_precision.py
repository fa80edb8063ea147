"""Weight-grad precision at long reductions: the f32 and bf16x3 GEMMs vs an
fp64 torch autograd reference on the GPU (FRCRN dec5 / enc1 geometry, full
4 s time axis, batch B)."""
import argparse, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip import functional as F

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
args = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
for name, tr, cin, cout, hw in [("dec5", True, 256, 128, (158, 403)), ("enc1", False, 128, 128, (158, 404))]:
    x = torch.randn(args.batch, cin, *hw, device=dev, dtype=torch.float64)
    wshape = (cin // 2, cout // 2, 5, 2) if tr else (cout // 2, cin // 2, 5, 2)
    wr = (torch.randn(wshape, device=dev, dtype=torch.float64) * 0.05).requires_grad_(True)
    wi = (torch.randn(wshape, device=dev, dtype=torch.float64) * 0.05).requires_grad_(True)
    # fp64 reference in the fused block-weight form
    if tr:
        wfull = torch.cat([torch.cat([wr, wi], 1), torch.cat([-wi, wr], 1)], 0)
        y = torch.nn.functional.conv_transpose2d(x, wfull, stride=(2, 1))
    else:
        wfull = torch.cat([torch.cat([wr, -wi], 1), torch.cat([wi, wr], 1)], 0)
        y = torch.nn.functional.conv2d(x, wfull, stride=(2, 1))
    gy = torch.randn_like(y)
    y.backward(gy)
    for math in ("f32", "bf16x3"):
        F.set_conv_math(math)
        w1 = wr.detach().float().requires_grad_(True)
        w2 = wi.detach().float().requires_grad_(True)
        xf = x.float().requires_grad_(True)
        yh = F.conv2d(xf, w1, w2, out_channels=cout, kernel=(5, 2), stride=(2, 1), transposed=tr)
        yh.backward(gy.float())
        torch.cuda.synchronize()
        e = lambda a, b: ((a.double() - b).norm() / b.norm()).item()
        print(f"{name} B={args.batch} M={y.shape[0]*y.shape[2]*y.shape[3] if not tr else x.shape[0]*hw[0]*hw[1]} "
              f"{math:6s} y {e(yh.detach(), y.detach()):.2e} dx {e(xf.grad, x.grad if x.grad is not None else xf.grad.double()):.2e} "
              f"dwr {e(w1.grad, wr.grad):.2e} dwi {e(w2.grad, wi.grad):.2e}", flush=True)
    F.set_conv_math("f32")
