"""The three-multiplication complex forward GEMM (gather_3m_kernel, SEHIP_GEMM_3M=1):
y_re = (xr + xi) Wr - xi (Wr + Wi), y_im = (xr + xi) Wr + xr (Wi - Wr), 3/4 of the
MFMA issues of the 4-product block GEMM (complex_nn.py:52-91's four real convs).

Bar: fp32-class, as the default f16x3 path — the forward output against the fp64
oracle at or below 1.25x the exact-fp32 MFMA path's own error (and < 1e-5), at the
FRCRN layer geometries with 64 complex outputs (encoder conv, decoder convT with its
stride-phase classes), for the decoder's joined input (complex_concat([x, skip]),
frcrn.py:93-101) against the fp64 conv of the materialised join, across operand
scales, and the whole FRCRN train step against the 4-product form."""
import pytest
import torch

from conftest import rel_l2
from test_gpu_conv_x3 import F16_VS_F32, LAYERS, _fp64_ref, _hip

pytestmark = pytest.mark.gpu

M3_LAYERS = [lay for lay in LAYERS if lay[3] == 128]   # 64 complex outputs


@pytest.fixture
def m3(monkeypatch):
    monkeypatch.setenv("SEHIP_GEMM_3M", "1")


@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", M3_LAYERS)
@pytest.mark.parametrize("scales", [(1.0, 1.0), (2.0 ** -40, 1.0), (2.0 ** 30, 1.0)])
def test_3m_forward_vs_fp64(name, tr, cin, cout, shape, stride, scales, gpu_device, monkeypatch):
    from sehip import functional as F
    m, x, gy, ref = _fp64_ref(name, tr, cin, cout, shape, stride, *scales)
    exact = _hip(F, m, x, gy, tr, stride, "f32")
    four = _hip(F, m, x, gy, tr, stride, "f16x3")
    monkeypatch.setenv("SEHIP_GEMM_3M", "1")
    three = _hip(F, m, x, gy, tr, stride, "f16x3")
    e32 = rel_l2(exact["y"].numpy(), ref["y"].numpy())
    e4 = rel_l2(four["y"].numpy(), ref["y"].numpy())
    e3 = rel_l2(three["y"].numpy(), ref["y"].numpy())
    print(f"{name} y: f32 {e32:.2e}  f16x3 4M {e4:.2e}  f16x3 3M {e3:.2e}")
    assert e3 < 1e-5 and e3 <= max(F16_VS_F32 * e32, 1e-7), (name, e3, e32)
    for k in ("dx", "dwr", "dwi"):   # the backward passes do not change
        assert torch.equal(three[k], four[k]), k


@pytest.mark.parametrize("xs,ss", [((2, 128, 17, 41), (2, 128, 17, 40)),    # time crop
                                   ((2, 128, 16, 41), (2, 128, 17, 40)),    # + frequency pad
                                   ((3, 128, 40, 21), (3, 128, 40, 21))])   # aligned, partial M-tile
def test_3m_joined_forward_vs_fp64(gpu_device, xs, ss, m3):
    from oracle.complex_nn import complex_concat
    from sehip import functional as F
    torch.manual_seed(1)
    x, s = torch.randn(xs, dtype=torch.float64), torch.randn(ss, dtype=torch.float64)
    cin, cout = 2 * xs[1], 128
    wr = torch.randn(cin // 2, cout // 2, 5, 2, dtype=torch.float64) * 0.05
    wi = torch.randn(cin // 2, cout // 2, 5, 2, dtype=torch.float64) * 0.05
    xa = x[..., :-1] if x.shape[-1] > s.shape[-1] else x
    if xa.shape[-2] < s.shape[-2]:
        xa = torch.nn.functional.pad(xa, (0, 0, 0, 1))
    j = complex_concat([xa, s], dim=1)
    wb = torch.cat([torch.cat([wr, wi], 1), torch.cat([-wi, wr], 1)], 0)   # (Cin, Cout) block
    ref = torch.nn.functional.conv_transpose2d(j, wb, stride=(2, 1))
    y = F.conv2d_joined(x.float().cuda(), s.float().cuda(), wr.float().cuda(), wi.float().cuda(),
                        out_channels=cout, kernel=(5, 2), stride=(2, 1), transposed=True)
    torch.cuda.synchronize()
    yc = y.double().cpu()
    assert yc.shape == ref.shape
    e3 = ((yc - ref).norm() / ref.norm()).item()
    ref32 = torch.nn.functional.conv_transpose2d(j.float(), wb.float(), stride=(2, 1)).double()
    e32 = ((ref32 - ref).norm() / ref.norm()).item()   # the CPU fp32 conv, for scale
    print(f"joined {xs}: 3M {e3:.2e}  CPU fp32 {e32:.2e}")
    assert e3 < 1e-6


def test_3m_frcrn_forward(gpu_device, monkeypatch):
    """FRCRN forward with every 64-output split-fp16 forward on the 3M form against the
    4-product form."""
    import paramfill
    from sehip.models import FRCRN

    def run():
        m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
        noisy, _ = (torch.from_numpy(t).cuda() for t in paramfill.structured_pair(2, 16000, seed=60))
        spec, wav = m(noisy)
        torch.cuda.synchronize()
        return spec.detach(), wav.detach()

    s0, w0 = run()
    monkeypatch.setenv("SEHIP_GEMM_3M", "1")
    s1, w1 = run()
    assert ((s1 - s0).norm() / s0.norm()).item() <= 1e-5
    assert ((w1 - w0).norm() / w0.norm()).item() <= 1e-5


def test_3m_frcrn_train_step_vs_fp64(gpu_device, m3):
    """The train-step golden with the 3M forward: output, loss, and every parameter
    gradient through the per-tensor fp64 gate of tests/test_gpu_models.py (the gradients of
    the CCBAM max / ReLU routing are ill-conditioned, so 3M and 4M are each compared with
    fp64, not with each other)."""
    from test_gpu_models import test_frcrn_train_step_golden
    test_frcrn_train_step_golden(gpu_device)
