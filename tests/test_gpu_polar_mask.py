"""se_polar_mask_fwd (the inference masks of DCUNet / DCCRN, ABI 9) against the reference's
own op sequences: DCUNet bounded_tanh (/root/reference/models/_1903_03107_dcunet.py:167-189)
and DCCRN 'E' (/root/reference/models/_2008_00264_dccrn.py:194-207). The kernel rounds every
intermediate to the storage type where the reference's tensors are rounded, in the same order
and without contraction; its sin / cos / tanh / atan2 are this toolchain's, which may differ from
torch's build in the last ulp, and the phase terms amplify such an ulp. So the gate is the
reference's own: against an fp64 evaluation of the formula, the fused pass's error is within
1.5x (+ a floor) of the torch op sequence's error in the same storage type."""
import pytest
import torch

from sehip import functional as F

pytestmark = pytest.mark.gpu


def _mag_phase(re, im):
    return torch.sqrt(re ** 2 + im ** 2 + 1e-8), torch.atan2(im, re)


def _ref(mr, mi, nr, ni, mode):
    n_mag, n_ph = _mag_phase(nr, ni)
    m_mag, m_ph = _mag_phase(mr, mi)
    if mode == 0:
        ph = n_ph + m_ph / m_mag
    else:
        ph = n_ph + torch.atan2(mi / m_mag, mr / m_mag)
    gain = n_mag * torch.tanh(m_mag)
    return torch.stack([gain * torch.cos(ph), gain * torch.sin(ph)], dim=1)


def _rms(a, b):
    return (a.double() - b.double()).pow(2).mean().sqrt().item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mode", [0, 1])
def test_polar_mask_matches_reference_ops(dtype, mode):
    g = torch.Generator(device="cuda").manual_seed(3 + mode)
    B, Fq, T = 3, 65, 77
    # strided planes as the models pass them: the mask trimmed out of a wider decoder
    # output, the noisy halves of one spectrum
    h = torch.randn(B, 2, Fq + 2, T + 3, device="cuda", generator=g)[:, :, :Fq, :T]
    spec = 3 * torch.randn(B, 2 * Fq, T, device="cuda", generator=g)
    if dtype != torch.float16:   # the atan2 / eps corners (1e-8 underflows in fp16)
        h[0, :, :2, :5] = 0
        spec[1, :3, :4] = 0
        spec[1, Fq:Fq + 3, :4] = 0
    h, spec = h.to(dtype), spec.to(dtype)
    mr, mi, nr, ni = h[:, 0], h[:, 1], spec[:, :Fq], spec[:, Fq:]
    with torch.no_grad():
        got = F.polar_mask_nograd(mr, mi, nr, ni, mode)
        want = _ref(mr, mi, nr, ni, mode)
        exact = _ref(*(t.double() for t in (mr, mi, nr, ni)), mode)
    assert got is not None and got.dtype == dtype and got.shape == (B, 2, Fq, T)
    assert torch.isfinite(got).all() and torch.isfinite(want).all()
    floor = 4 * torch.finfo(dtype).eps * exact.abs().max().item() / 64
    e_got, e_ref = _rms(got, exact), _rms(want, exact)
    assert e_got <= 1.5 * e_ref + floor, (e_got, e_ref, floor)


def test_polar_mask_declines_a_training_forward():
    m = torch.randn(2, 5, 7, device="cuda", requires_grad=True)
    n = torch.randn(2, 5, 7, device="cuda")
    assert F.polar_mask_nograd(m, m, n, n, 0) is None
    with torch.no_grad():
        assert F.polar_mask_nograd(m, m, n, n, 0) is not None


def _ref_grads(mr, mi, nr, ni, mode, g):
    a, c = mr.detach().clone().requires_grad_(True), mi.detach().clone().requires_grad_(True)
    out = _ref(a, c, nr, ni, mode)
    out.backward(g.to(out.dtype))
    return out.detach(), a.grad, c.grad


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", [0, 1])
def test_polar_mask_backward_matches_autograd(dtype, mode):
    """_PolarMask's backward (se_polar_mask_bwd) against autograd of the reference op sequence:
    against fp64 autograd, its gradient error is within 1.5x (+ a floor) of torch's own in the
    same storage type. Mask magnitudes >= 0.3 keep the phase terms (m_ph / m_mag,
    atan2(v, u)) well conditioned, so the comparison measures the arithmetic, not the chaos."""
    g = torch.Generator(device="cuda").manual_seed(11 + mode)
    B, Fq, T = 2, 33, 51
    r = 0.3 + torch.rand(B, Fq, T, device="cuda", generator=g)
    th = 2 * torch.pi * torch.rand(B, Fq, T, device="cuda", generator=g)
    mr, mi = (r * torch.cos(th)).to(dtype), (r * torch.sin(th)).to(dtype)
    spec = (2 * torch.randn(B, 2, Fq, T, device="cuda", generator=g)).to(dtype)
    nr, ni = spec[:, 0], spec[:, 1]
    gout = torch.randn(B, 2, Fq, T, device="cuda", generator=g).to(dtype)
    a, c = mr.clone().requires_grad_(True), mi.clone().requires_grad_(True)
    n0 = F.POLAR_MASK_CALLS[0]
    out = F.polar_mask(a, c, nr, ni, mode)
    assert out is not None and F.POLAR_MASK_CALLS[0] == n0 + 1
    out.backward(gout)
    want = _ref_grads(mr, mi, nr, ni, mode, gout)
    exact = _ref_grads(*(t.double() for t in (mr, mi, nr, ni)), mode, gout.double())
    for name, x, w, e in zip(("out", "dmr", "dmi"), (out.detach(), a.grad, c.grad), want, exact):
        floor = 4 * torch.finfo(dtype).eps * e.abs().max().item() / 64
        e_got, e_ref = _rms(x, e), _rms(w, e)
        assert e_got <= 1.5 * e_ref + floor, (name, e_got, e_ref, floor)


def test_models_route_inference_through_the_fused_mask():
    """DCUNet: a no-grad forward runs the fused mask, a grad-enabled one the reference ops.
    DCCRN ('E'): both run the differentiable fused op; with it switched off the reference ops.
    The two agree to fp32 rounding (rel-L2 1e-5, north_star's 1e-4 bar). Inputs: the variant
    goldens' waveforms (lengths the models' grids accept)."""
    from conftest import golden
    from sehip import models as M
    torch.manual_seed(0)
    x = torch.from_numpy(golden("variant_dcunet10")["x"]).cuda()
    m = M.DCUNet("dcunet10", 512, 128, 512).cuda().eval()
    n0 = F.POLAR_MASK_CALLS[0]
    with torch.no_grad():
        est_f, wav_f = m(x)
    assert F.POLAR_MASK_CALLS[0] == n0 + 1
    est_r, wav_r = m(x)   # grad enabled, parameters require grad: the reference ops
    assert F.POLAR_MASK_CALLS[0] == n0 + 1
    pairs = [(est_f, est_r.detach()), (wav_f, wav_r.detach())]
    x = torch.from_numpy(golden("variant_dccrn_bi")["x"]).cuda()
    m = M.DCCRN("dccrn-CL", 400, 100, 512, bidirectional=True).cuda().eval()
    n0 = F.POLAR_MASK_CALLS[0]
    est_f, wav_f = m(x)
    assert F.POLAR_MASK_CALLS[0] == n0 + 1
    polar, stored = F.polar_mask, F.polar_mask_stored
    try:
        F.polar_mask = lambda *a, **k: None
        F.polar_mask_stored = lambda *a, **k: None
        est_r, wav_r = m(x)
    finally:
        F.polar_mask, F.polar_mask_stored = polar, stored
    pairs += [(est_f.detach(), est_r.detach()), (wav_f.detach(), wav_r.detach())]
    for a, b in pairs:
        rel = ((a.double() - b.double()).norm() / b.double().norm()).item()
        assert rel <= 1e-5, rel


def test_polar_mask_backward_fp16(gpu_device):
    """The fp16 backward (DCCRN .half() training) against autograd of the reference op
    sequence, as the fp32 / bf16 cases above (round-5 advice)."""
    test_polar_mask_backward_matches_autograd(torch.float16, 1)
    test_polar_mask_backward_matches_autograd(torch.float16, 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_polar_mask_zero_mask_nan_pattern(gpu_device, dtype):
    """Mask elements at (0, 0) and near zero (DCCRN 'E', the mode that trains): the kernel's
    backward has torch's finite / non-finite pattern. torch's atan2 backward is 0 where
    x^2 + y^2 == 0 (not NaN), so at the origin the fp32 gradient is finite (0 from the phase
    path); in fp16 the 1e-8 of the magnitude underflows, the forward itself is NaN at the
    origin, and so are both gradients."""
    g = torch.Generator(device="cuda").manual_seed(17)
    B, Fq, T = 1, 9, 16
    mr = torch.randn(B, Fq, T, device="cuda", generator=g).to(dtype)
    mi = torch.randn(B, Fq, T, device="cuda", generator=g).to(dtype)
    mr[0, 0, :4] = 0
    mi[0, 0, :4] = 0
    mr[0, 1, :4] = torch.tensor([1e-3, -1e-3, 2e-3, 0.0]).to(dtype)   # near zero, representable in both
    mi[0, 1, :4] = torch.tensor([0.0, 1e-3, -2e-3, 1e-3]).to(dtype)
    spec = torch.randn(B, 2, Fq, T, device="cuda", generator=g).to(dtype)
    nr, ni = spec[:, 0], spec[:, 1]
    gout = torch.randn(B, 2, Fq, T, device="cuda", generator=g).to(dtype)
    a, c = mr.clone().requires_grad_(True), mi.clone().requires_grad_(True)
    F.polar_mask(a, c, nr, ni, 1).backward(gout)
    _, ra, rc = _ref_grads(mr, mi, nr, ni, 1, gout)
    for got, want in ((a.grad, ra), (c.grad, rc)):
        diff = torch.isfinite(got) != torch.isfinite(want)
        assert not diff.any(), (diff.nonzero()[:6].tolist(), got[diff][:6].tolist(), want[diff][:6].tolist(),
                                mr[diff][:6].tolist(), mi[diff][:6].tolist())
    assert torch.isfinite(a.grad[0, 0, :4]).all() == (dtype == torch.float32)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_polar_mask_stored_equals_pad_trim_form(gpu_device, dtype):
    """DCCRN's mask from the stored decoder output (ABI 10, m_row0 = 1): the top zero row
    (F.pad, dccrn.py:172) and the trailing-frame trim (:180-182) folded into the kernels;
    values and the decoder-output gradient bit-identical to pad + slice + polar_mask."""
    g = torch.Generator(device="cuda").manual_seed(21)
    B, Fq, T = 2, 17, 30
    dec = (0.3 + torch.rand(B, 2, Fq - 1, T + 1, device="cuda", generator=g)).to(dtype)
    spec = torch.randn(B, 2, Fq, T, device="cuda", generator=g).to(dtype)
    nr, ni = spec[:, 0], spec[:, 1]
    gout = torch.randn(B, 2, Fq, T, device="cuda", generator=g).to(dtype)
    d1 = dec.clone().requires_grad_(True)
    out1 = F.polar_mask_stored(d1, nr, ni, 1, row0=1)
    out1.backward(gout)
    d2 = dec.clone().requires_grad_(True)
    h = torch.nn.functional.pad(d2, (0, 0, 1, 0))
    out2 = F.polar_mask(h[:, 0, :, :T], h[:, 1, :, :T], nr, ni, 1)
    out2.backward(gout)
    assert torch.equal(out1, out2)
    assert torch.equal(d1.grad, d2.grad)
    assert torch.count_nonzero(d1.grad[..., T:]) == 0
