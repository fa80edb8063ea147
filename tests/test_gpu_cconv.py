"""GPU parity: fused complex conv / convT implicit GEMM vs reference goldens
and vs the oracle's four-real-conv form at FRCRN layer shapes (fp32, 1e-5)."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2
import paramfill
from oracle import complex_nn as O_cnn

pytestmark = pytest.mark.gpu

CONV_CASES = [
    ("enc", False, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
    ("padbias", False, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=True)),
    ("k7", False, 4, 2, 7, dict(padding=3, bias=False)),
    ("dec", True, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
    ("dccrn_dec", True, 8, 6, (5, 2), dict(stride=(2, 1), padding=(2, 0), output_padding=(1, 0), bias=True)),
    ("dcunet_dec", True, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=False)),
]


def _run(F, m, x, gy, transposed, kw):
    wr = m.real_conv.weight.detach().cuda().requires_grad_(True)
    wi = m.imag_conv.weight.detach().cuda().requires_grad_(True)
    br = bi = None
    if m.real_conv.bias is not None:
        br = m.real_conv.bias.detach().cuda().requires_grad_(True)
        bi = m.imag_conv.bias.detach().cuda().requires_grad_(True)
    xg = x.cuda().requires_grad_(True)
    y = F.conv2d(xg, wr, wi, br, bi, out_channels=2 * m.real_conv.out_channels,
                 kernel=m.real_conv.kernel_size, stride=kw.get("stride", 1),
                 padding=kw.get("padding", 0), output_padding=kw.get("output_padding", 0),
                 transposed=transposed)
    y.backward(gy.cuda())
    torch.cuda.synchronize()
    out = dict(y=y.detach().cpu(), dx=xg.grad.cpu(), dwr=wr.grad.cpu(), dwi=wi.grad.cpu())
    if br is not None:
        out.update(dbr=br.grad.cpu(), dbi=bi.grad.cpu())
    return out


@pytest.mark.parametrize("i,case", list(enumerate(CONV_CASES)))
def test_conv_golden(i, case, gpu_device):
    from sehip import functional as F
    g = golden("cconv")
    name, tr, cin, cout, k, kw = case
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, k, **kw), seed=i)
    r = _run(F, m, torch.from_numpy(g[f"{name}_x"]), torch.from_numpy(g[f"{name}_gy"]), tr, kw)
    for key in ("y", "dx", "dwr", "dwi") + (("dbr", "dbi") if f"{name}_dbr" in g else ()):
        assert rel_l2(r[key].numpy(), g[f"{name}_{key}"]) < 1e-5, (name, key)


def test_real_conv_golden(gpu_device):
    from sehip import functional as F
    g = golden("cconv")
    m = paramfill.fill_(torch.nn.Conv2d(16, 2, (1, 2), bias=False), seed=9)
    w = m.weight.detach().cuda().requires_grad_(True)
    x = torch.from_numpy(g["real_x"]).cuda().requires_grad_(True)
    y = F.conv2d(x, w, out_channels=2, kernel=(1, 2))
    y.backward(torch.from_numpy(g["real_gy"]).cuda())
    assert rel_l2(y.detach().cpu().numpy(), g["real_y"]) < 1e-5
    assert rel_l2(x.grad.cpu().numpy(), g["real_dx"]) < 1e-5
    assert rel_l2(w.grad.cpu().numpy(), g["real_dw"]) < 1e-5


# FRCRN layer geometries at reduced batch/time (frcrn.py:62-102)
FRCRN_LAYERS = [
    ("enc0", False, 2, 128, (2, 2, 320, 41)),
    ("enc1", False, 128, 128, (2, 128, 158, 41)),
    ("enc5", False, 128, 128, (2, 128, 7, 41)),
    ("dec0", True, 256, 128, (2, 256, 2, 40)),
    ("dec4", True, 256, 128, (2, 256, 77, 40)),
    ("dec5", True, 256, 128, (2, 256, 158, 40)),
]


# fp32-class modes at 1e-5 against the fp64 oracle; bf16x3 (two-term split bf16) at 3e-5
MATH_TOL = {"f32": 1e-5, "f16x3": 1e-5, "bf16x6": 1e-5, "bf16x3": 3e-5}


@pytest.mark.parametrize("math", sorted(MATH_TOL))
@pytest.mark.parametrize("name,tr,cin,cout,shape", FRCRN_LAYERS)
def test_frcrn_layer_vs_oracle(name, tr, cin, cout, shape, math, gpu_device):
    """Every FRCRN encoder/decoder layer shape, every pass, each MFMA form
    against the fp64 oracle (bf16x6 has no weight-grad kernel: f32 there)."""
    from sehip import functional as F
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, (5, 2), stride=(2, 1), bias=False), seed=7).double()
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=gen, dtype=torch.float64)
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    gy = torch.randn(yo.shape, generator=gen, dtype=torch.float64)
    yo.backward(gy)
    ref = dict(y=yo.detach().numpy(), dx=xo.grad.numpy(), dwr=m.real_conv.weight.grad.numpy().copy(),
               dwi=m.imag_conv.weight.grad.numpy().copy())
    prev = F.get_conv_math()
    try:
        F.set_conv_math(math if math != "bf16x6" else "fwd=bf16x6,data=bf16x6,weight=f32")
        r = _run(F, m.float(), x.float(), gy.float(), tr, dict(stride=(2, 1)))
    finally:
        F.set_conv_math(prev)
    tol = MATH_TOL[math]
    errs = {k: rel_l2(r[k].numpy(), ref[k]) for k in ("y", "dwr", "dwi") + (("dx",) if name != "enc0" else ())}
    print(name, math, {k: f"{v:.2e}" for k, v in errs.items()})
    for k, e in errs.items():
        assert e < tol, (name, math, k, e)


@pytest.mark.parametrize("input_pad", [(1, 0, 0, 0), (2, 1, 1, 3), (0, 3, 2, 0)])
def test_input_pad_folded_into_conv(input_pad, gpu_device):
    """ComplexConv2d(x, input_pad) == oracle conv of F.pad(x, input_pad): the
    causal pad of FRCRN's encoder blocks (frcrn.py:28-30) as asymmetric conv
    padding, forward and all three backward passes."""
    from sehip.complex_nn import ComplexConv2d
    torch.manual_seed(11)
    ref = paramfill.fill_(O_cnn.ComplexConv2d(16, 12, (5, 2), stride=(2, 1), padding=(1, 0), bias=True), seed=3)
    mod = ComplexConv2d(16, 12, (5, 2), stride=(2, 1), padding=(1, 0), bias=True)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 16, 21, 13)
    xr = x.clone().requires_grad_(True)
    yr = ref(torch.nn.functional.pad(xr, input_pad))
    gy = torch.randn_like(yr)
    (yr * gy).sum().backward()
    mod = mod.to(gpu_device)
    xd = x.to(gpu_device).requires_grad_(True)
    yd = mod(xd, input_pad)
    assert yd.shape == yr.shape
    assert rel_l2(yd.detach().cpu().numpy(), yr.detach().numpy()) < 1e-5
    (yd * gy.to(gpu_device)).sum().backward()
    assert rel_l2(xd.grad.cpu().numpy(), xr.grad.numpy()) < 1e-5
    rp = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert rel_l2(p.grad.cpu().numpy(), rp[n].grad.numpy()) < 1e-5, n


# real-weight (nn.Conv2d / nn.ConvTranspose2d) geometries of CRN / CARN (real_conv2d),
# against torch's CPU autograd in fp32; output_padding in either dim
REAL_CASES = [
    ("crn_enc", False, 16, 32, (2, 3), dict(stride=(1, 2), padding=(1, 0)), (2, 16, 6, 39)),
    ("crn_dec3", True, 64, 16, (2, 3), dict(stride=(1, 2), output_padding=(0, 1)), (2, 64, 6, 19)),
    ("crn_dec1", True, 256, 64, (2, 3), dict(stride=(1, 2)), (2, 256, 5, 9)),
    ("carn_dec", True, 64, 32, (1, 3), dict(stride=(2, 1), padding=(0, 1), output_padding=(1, 0)), (2, 64, 9, 11)),
    ("carn_att", False, 32, 64, (3, 3), dict(padding=(1, 1)), (2, 32, 17, 11)),
    # CRN's decoder at the golden 1 s input (T = 101 frames)
    ("crn_dec2_full", True, 128, 32, (2, 3), dict(stride=(1, 2)), (2, 128, 101, 19)),
    ("crn_dec3_full", True, 64, 16, (2, 3), dict(stride=(1, 2), output_padding=(0, 1)), (2, 64, 101, 39)),
    ("crn_dec4_full", True, 32, 1, (2, 3), dict(stride=(1, 2)), (2, 32, 101, 80)),
    ("crn_enc1_full", False, 16, 32, (2, 3), dict(stride=(1, 2), padding=(1, 0)), (2, 16, 101, 80)),
]


@pytest.mark.parametrize("case", REAL_CASES, ids=[c[0] for c in REAL_CASES])
def test_real_conv_geometries_vs_torch(case, gpu_device):
    from sehip import functional as F
    from sehip.complex_nn import real_conv2d
    name, tr, cin, cout, k, kw, shape = case
    cls = torch.nn.ConvTranspose2d if tr else torch.nn.Conv2d
    torch.manual_seed(7)
    m = cls(cin, cout, k, bias=True, **kw)
    x = torch.randn(shape)
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    gy = torch.randn(yo.shape)
    yo.backward(gy)
    prev = F.get_conv_math()
    try:
        F.set_conv_math("f32")
        mc = cls(cin, cout, k, bias=True, **kw)
        mc.load_state_dict(m.state_dict())
        mc = mc.cuda()
        xg = x.cuda().requires_grad_(True)
        y = real_conv2d(mc, xg)
        y.backward(gy.cuda())
    finally:
        F.set_conv_math(prev)
    assert y.shape == yo.shape
    assert rel_l2(y.detach().cpu().numpy(), yo.detach().numpy()) < 1e-5, (name, "y")
    assert rel_l2(xg.grad.cpu().numpy(), xo.grad.numpy()) < 1e-5, (name, "dx")
    assert rel_l2(mc.weight.grad.cpu().numpy(), m.weight.grad.numpy()) < 1e-5, (name, "dw")
    assert rel_l2(mc.bias.grad.cpu().numpy(), m.bias.grad.numpy()) < 1e-5, (name, "db")
