"""Diagnostic: CBN forward from conv-epilogue moment rows vs the CBN's own pass vs fp64.
python tools/mom_diag.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement_amd"))
import torch  # noqa: E402

from sehip import functional as F  # noqa: E402
from sehip.complex_nn import ComplexBatchNorm2d  # noqa: E402


def ref_cbn(y, bn):
    yd = y.double()
    Cc = y.shape[1] // 2
    yr, yi = yd[:, :Cc], yd[:, Cc:]
    mr, mi = yr.mean((0, 2, 3)), yi.mean((0, 2, 3))
    cr, ci = yr - mr[None, :, None, None], yi - mi[None, :, None, None]
    vrr = (cr * cr).mean((0, 2, 3)) + bn.eps
    vri = (cr * ci).mean((0, 2, 3))
    vii = (ci * ci).mean((0, 2, 3)) + bn.eps
    s = (vrr * vii - vri * vri).sqrt()
    t = (vrr + vii + 2 * s).sqrt()
    r = 1 / (s * t)
    urr, uii, uri = (s + vii) * r, (s + vrr) * r, -vri * r
    wrr, wri, wii = bn.Wrr.double(), bn.Wri.double(), bn.Wii.double()
    zrr, zri = wrr * urr + wri * uri, wrr * uri + wri * uii
    zir, zii = wri * urr + wii * uri, wri * uri + wii * uii
    e = lambda v: v[None, :, None, None]  # noqa: E731
    outr = e(zrr) * cr + e(zri) * ci + e(bn.Br.double())
    outi = e(zir) * cr + e(zii) * ci + e(bn.Bi.double())
    return torch.cat([outr, outi], 1), (mr, mi)


def main():
    dev = torch.device("cuda")
    torch.manual_seed(4)
    x = torch.randn(2, 128, 33, 37, device=dev) * 2 + 0.5
    wr = torch.randn(64, 64, 5, 2, device=dev) * 0.05
    wi = torch.randn(64, 64, 5, 2, device=dev) * 0.05
    kw = dict(out_channels=128, kernel=(5, 2), stride=(2, 1), padding=(2, 0))
    for rg in (False, True):
        for emit in (True, False):
            bn = ComplexBatchNorm2d(128).to(dev).train()
            with torch.no_grad():
                bn.Wrr.add_(0.3)
                bn.Br.add_(0.1)
            xa = x.clone().requires_grad_(rg)
            with F.emit_moments(emit):
                y = F.conv2d(xa, wr, wi, **kw)
            e = F.moments_take(y) if emit else None
            if e is not None:
                F.moments_put(y, *e)
                buf, rows = e
                Cc = 64
                part = buf[:Cc * rows * 40].view(torch.float64).view(Cc, rows, 5).sum(1)
                yd = y.detach().double()
                print(f"  rows={rows} sum_r got {part[:3, 0].tolist()} ref {yd[:, :Cc].sum((0, 2, 3))[:3].tolist()}")
            z = bn.forward_act(y, 0, 0.2)
            torch.cuda.synchronize()
            zr, (mr, mi) = ref_cbn(y.detach(), bn)
            err = ((z.double() - zr).norm() / zr.norm()).item()
            print(f"requires_grad={rg} emit={emit}: z vs fp64 {err:.3e}; RMr {bn.RMr[:3].tolist()} "
                  f"ref {(0.1 * mr[:3]).tolist()}")


if __name__ == "__main__":
    main()
