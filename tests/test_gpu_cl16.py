"""CL16 operands (ABI 7): the decoder's joined-conv inputs written pre-split by their
producers (ComplexBN forward's y_packed, CCBAM's out_packed) and read by the joined
weight-grad GEMM as its D operand (se_conv2d_desc.x_packed / x2_packed), replacing
the fp32 gather + split of the reference formulation's conv backward
(frcrn.py:93-101, complex_nn.py:80-91).

The CL16 form of a tensor t with bound A is the SE_MATH_F16X3 split of t * s,
s = 2^(14 - e), max|t| <= A < 2^e: hi = fp16(t s), lo = fp16(t s - hi), channels
innermost, [2][B][H][W][C]. Layout and producers are checked bit-exactly against a
torch restatement; the weight-grad against its fp32-operand form (bit-identical
when both sources share one bound) and against fp64 (each source its own bound).
"""
import copy
import ctypes

import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _cl16_on(monkeypatch):
    """The Python host writes the copies only under SEHIP_CL16=1 (opt-in: measured slower
    at the bench step); the library paths are tested with it on."""
    monkeypatch.setenv("SEHIP_CL16", "1")


def _cl16_ref(t: torch.Tensor, amax: torch.Tensor) -> torch.Tensor:
    """Torch restatement of the CL16 form (fp16 [2, B, H, W, C])."""
    a = float(amax.item())
    e = int(np.frexp(np.float32(a))[1]) if a > 0 else -126   # a < 2^e
    e = max(-100, min(100, e))
    v = t.float().permute(0, 2, 3, 1) * float(2.0 ** (14 - e))
    hi = v.half()
    lo = (v - hi.float()).half()
    return torch.stack([hi, lo])


def _pack(t, amax):
    from sehip import _native as N
    B, C, H, W = t.shape
    out = torch.empty(2 * t.numel(), dtype=torch.float16, device=t.device)
    N.check(N.lib().se_pack_cl16(t.data_ptr(), B, C, H, W, amax.data_ptr(), out.data_ptr(), N.stream_of(t)),
            "se_pack_cl16")
    return out


def test_pack_cl16_layout(gpu_device):
    torch.manual_seed(0)
    t = torch.randn(2, 64, 9, 37, device=gpu_device) * 3
    t[0, 3, 2, 5] = 0.0
    amax = t.abs().max().reshape(1) * 1.5
    got = _pack(t, amax).view(2, 2, 9, 37, 64)
    assert torch.equal(got, _cl16_ref(t, amax))


def test_cbn_forward_writes_cl16_copy(gpu_device):
    """se_cbn_fwd's y_packed = the CL16 form of its own y with its own y_amax bound."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d
    torch.manual_seed(1)
    bn = ComplexBatchNorm2d(128).cuda().train()
    bn2 = copy.deepcopy(bn)
    x = torch.randn(3, 128, 11, 41, device=gpu_device, requires_grad=True) * 2 + 0.5
    n0 = F.CL16_CALLS[0]
    y = bn.forward_act(x, F.ACT_LEAKY, 0.2, pack=True)
    assert F.CL16_CALLS[0] == n0 + 1
    buf, ya = F.cl16_get(y)
    assert ya is F.amax_get(y)
    got = buf.view(2, 3, 11, 41, 128)
    assert torch.equal(got, _cl16_ref(y.detach(), ya))
    # and the fp32 y is the one the kernel without the copy writes
    assert torch.equal(y.detach(), bn2.forward_act(x, F.ACT_LEAKY, 0.2).detach())


def test_ccbam_writes_cl16_copy(gpu_device):
    """se_ccbam_apply's out_packed = the CL16 form of out with the bound max|x| + 1."""
    import paramfill
    from sehip import functional as F
    from sehip.ccbam import CCBAM
    torch.manual_seed(2)
    m = paramfill.fill_(CCBAM(128, 16), seed=3).cuda().train()
    x = (torch.randn(2, 128, 9, 37, device=gpu_device) * 2).requires_grad_(True)
    F.amax_put(x, x.detach().abs().max().reshape(1) * 1.01)
    out = m(x, pack=True)
    buf, oa = F.cl16_get(out)
    assert torch.equal(buf.view(2, 2, 9, 37, 128), _cl16_ref(out.detach(), oa))
    assert torch.equal(out.detach(), m(x).detach())


def _joined_wgrad(x, s, gy, x_amax, x2_amax=None, xpk=None, spk=None, gy_amax=None):
    """se_conv2d_bwd_weight_joined of the FRCRN decoder convT (5, 2) / (2, 1) over
    complex_join(x, s), f16x3; CL16 D operands when xpk / spk are given."""
    from sehip import functional as F, _native as N
    B, C, F_, T = s.shape
    d = F.conv_desc((B, 2 * C, F_, T), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
    d.math = F._MATH_CODES["f16x3"]
    lib = N.lib()
    ws = torch.empty(lib.se_conv2d_workspace_size(ctypes.byref(d)), dtype=torch.uint8, device=x.device)
    dwr = torch.empty(C, 64, 5, 2, device=x.device)
    dwi = torch.empty_like(dwr)
    d.x_amax = x_amax.data_ptr()
    d.dy_amax = None if gy_amax is None else gy_amax.data_ptr()
    if xpk is not None:
        d.x_packed, d.x2_packed, d.x2_amax = spk.data_ptr(), xpk.data_ptr(), x2_amax.data_ptr()
    rc = lib.se_conv2d_bwd_weight_joined(ctypes.byref(d), x.data_ptr(), x.shape[2], x.shape[3], s.data_ptr(),
                                         gy.data_ptr(), dwr.data_ptr(), dwi.data_ptr(), None, None, ws.data_ptr(),
                                         ws.numel(), N.stream_of(x))
    return rc, dwr, dwi


SHAPES = [((2, 128, 17, 41), (2, 128, 17, 40)),     # dec3-like: time crop
          ((2, 128, 77, 41), (2, 128, 78, 40)),     # dec5-like: crop + freq pad
          ((3, 128, 7, 21), (3, 128, 7, 21))]       # aligned, several items per m-split


def _operands(xs, ss, gx, gs, seed):
    gen = torch.Generator().manual_seed(seed)
    x = (torch.randn(xs, generator=gen, dtype=torch.float64) * gx).float().cuda()
    s = (torch.randn(ss, generator=gen, dtype=torch.float64) * gs).float().cuda()
    B, C, F_, T = ss
    gy = torch.randn(B, 128, 2 * F_ + 3, T + 1, generator=gen, dtype=torch.float64).float().cuda()
    return x, s, gy


@pytest.mark.parametrize("xs,ss", SHAPES)
def test_joined_wgrad_cl16_bit_identical_with_one_bound(gpu_device, xs, ss):
    """x and s packed with the same (joint) bound: the CL16 weight-grad stages exactly
    the hi / lo planes the fp32 form splits in registers, over the same m-splits and
    K order, so dWr / dWi are bit-identical."""
    x, s, gy = _operands(xs, ss, 1.0, 3.0, 7)
    joint = torch.maximum(x.abs().max(), s.abs().max()).reshape(1)
    rc0, wr0, wi0 = _joined_wgrad(x, s, gy, joint)
    rc1, wr1, wi1 = _joined_wgrad(x, s, gy, joint, joint, _pack(x, joint), _pack(s, joint))
    torch.cuda.synchronize()
    assert rc0 == 0 and rc1 == 0
    assert torch.equal(wr0, wr1) and torch.equal(wi0, wi1)


@pytest.mark.parametrize("xs,ss", SHAPES[:2])
@pytest.mark.parametrize("gx,gs", [(1.0, 1.0), (2.0 ** -12, 1.0), (1.0, 2.0 ** -12)])
def test_joined_wgrad_cl16_vs_fp64(gpu_device, xs, ss, gx, gs):
    """Each source with its own bound (as the producers write them) against the fp64
    oracle's weight gradients (frcrn.py:93-101): at or below the exact fp32 MFMA path's
    error, also when x and s differ by 2^12 in level (a joint scale would leave the
    quieter source 12 bits fewer)."""
    import paramfill
    from oracle import complex_nn as O_cnn
    from test_gpu_join import _ref
    x, s, gy = _operands(xs, ss, gx, gs, 11)
    m = paramfill.fill_(O_cnn.ComplexConvTranspose2d(256, 128, (5, 2), stride=(2, 1), bias=False), seed=4).double()
    y = m(_ref(x.double().cpu(), s.double().cpu()))
    assert y.shape == gy.shape
    y.backward(gy.double().cpu())
    ref = (m.real_conv.weight.grad, m.imag_conv.weight.grad)
    xa, sa = x.abs().max().reshape(1), s.abs().max().reshape(1)
    rc, wr, wi = _joined_wgrad(x, s, gy, sa, xa, _pack(x, xa), _pack(s, sa))
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math("f32")
    try:   # the exact fp32 MFMA path (materialised join) as the bar
        xg, sg = x.clone(), s.clone()
        wrr = m.real_conv.weight.detach().float().cuda().requires_grad_(True)
        wii = m.imag_conv.weight.detach().float().cuda().requires_grad_(True)
        y32 = F.conv2d_joined(xg, sg, wrr, wii, out_channels=128, kernel=(5, 2), stride=(2, 1), transposed=True)
        y32.backward(gy)
    finally:
        F.set_conv_math(prev)
    torch.cuda.synchronize()
    assert rc == 0
    for got, f32, r in ((wr, wrr.grad, ref[0]), (wi, wii.grad, ref[1])):
        e, e32 = rel_l2(got.cpu().numpy(), r.numpy()), rel_l2(f32.cpu().numpy(), r.numpy())
        print(f"{xs} gains {gx:g}/{gs:g}: cl16 {e:.2e} exact-fp32 {e32:.2e}")
        assert e < max(1.25 * e32, 2e-7), (e, e32)


def test_joined_wgrad_cl16_refusals(gpu_device):
    """Only the joined split-fp16 weight-grad reads CL16; everything else refuses before
    launching (SE_E_UNSUPPORTED), and one source alone is refused too."""
    from sehip import functional as F, _native as N
    x, s, gy = _operands(*SHAPES[0], 1.0, 1.0, 3)
    a = torch.ones(1, device=gpu_device) * 8
    pk = _pack(x, a)
    B, C, F_, T = s.shape
    d = F.conv_desc((B, 2 * C, F_, T), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
    lib = N.lib()
    ws = torch.empty(lib.se_conv2d_workspace_size(ctypes.byref(d)), dtype=torch.uint8, device=gpu_device)
    dw = torch.empty(C, 64, 5, 2, device=gpu_device)
    d.x_amax, d.x2_amax, d.x2_packed = a.data_ptr(), a.data_ptr(), pk.data_ptr()   # x_packed missing
    for math in ("f16x3", "bf16x3"):
        d.math = F._MATH_CODES[math]
        rc = lib.se_conv2d_bwd_weight_joined(ctypes.byref(d), x.data_ptr(), x.shape[2], x.shape[3], s.data_ptr(),
                                             gy.data_ptr(), dw.data_ptr(), dw.data_ptr(), None, None, ws.data_ptr(),
                                             ws.numel(), N.stream_of(x))
        assert rc == -3, (math, rc)
    d.x_packed, d.math = pk.data_ptr(), F._MATH_CODES["f16x3"]   # the forward never reads CL16
    y = torch.empty(B, 128, 2 * F_ + 3, T + 1, device=gpu_device)
    rc = lib.se_conv2d_fwd_joined(ctypes.byref(d), x.data_ptr(), x.shape[2], x.shape[3], s.data_ptr(), dw.data_ptr(),
                                  dw.data_ptr(), None, None, y.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_of(x))
    assert rc == -3


def test_frcrn_train_step_reads_cl16(gpu_device):
    """In an FRCRN training step the decoder blocks' CBN and the CCBAM gates write the
    CL16 copies and the joined weight-grads of decoder layers 1-5 read them (layer 0's
    x is the LSTM output, which has none); the gradients still pass the fp64 gate of
    test_frcrn_train_step_golden (which runs this same path)."""
    import paramfill
    from sehip import functional as F, models as M
    from sehip.losses import SI_SNR_loss, pad_or_truncate_wav
    noisy, clean = paramfill.structured_pair(2, 16000, seed=4)
    m = paramfill.fill_(M.FRCRN(), seed=6).cuda().train()
    r0 = F.CL16_CALLS[1]
    _, wav = m(torch.from_numpy(noisy).cuda())
    c = torch.from_numpy(clean).cuda()
    SI_SNR_loss(pad_or_truncate_wav(wav, c), c).backward()
    torch.cuda.synchronize()
    assert F.CL16_CALLS[1] - r0 == 5
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())


def test_frcrn_train_step_cl16_matches_fp32_operands(gpu_device, monkeypatch):
    """SEHIP_CL16=0 (the default: the weight-grads split their fp32 D operand in the loop)
    vs the CL16 copies: identical forward outputs and data gradients (the copies do not
    touch them); the joined weight gradients differ only by the per-source scale of x and
    s (each split against its own bound instead of the joint one), within 1e-6."""
    import paramfill
    from sehip import models as M
    from sehip.losses import SI_SNR_loss, pad_or_truncate_wav
    noisy, clean = paramfill.structured_pair(2, 16000, seed=8)
    res = []
    for v in ("0", "1"):
        monkeypatch.setenv("SEHIP_CL16", v)
        m = paramfill.fill_(M.FRCRN(), seed=9).cuda().train()
        _, wav = m(torch.from_numpy(noisy).cuda())
        c = torch.from_numpy(clean).cuda()
        SI_SNR_loss(pad_or_truncate_wav(wav, c), c).backward()
        torch.cuda.synchronize()
        res.append((wav.detach(), {n: p.grad.detach() for n, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for n, g0 in res[0][1].items():
        g1 = res[1][1][n]
        e = ((g1 - g0).norm() / (g0.norm() + 1e-30)).item()
        assert e < 1e-6 or torch.equal(g0, g1), (n, e)
