"""se_complex_join(_bwd) (the FRCRN decoder's align + complex_concat,
frcrn.py:93-100) against the reference formulation on the CPU: forward and
both gradients must be bit-identical (pure data movement)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, s):
    from oracle.complex_nn import complex_concat
    if x.shape[-1] > s.shape[-1]:
        x = x[..., :-1]
    if x.shape[-2] < s.shape[-2]:
        x = torch.nn.functional.pad(x, (0, 0, 0, 1))
    return complex_concat([x, s], dim=1)


@pytest.mark.parametrize("xs,ss", [
    ((2, 8, 7, 14), (2, 6, 7, 13)),      # time crop only (every decoder layer)
    ((2, 8, 6, 14), (2, 8, 7, 13)),      # crop + freq pad (157 -> 158 in FRCRN)
    ((3, 4, 5, 9), (3, 4, 5, 9)),        # already aligned (first decoder layer)
    ((1, 2, 4, 10), (1, 6, 5, 10)),      # pad only
])
def test_complex_join_matches_reference(gpu_device, xs, ss):
    from sehip import functional as F
    torch.manual_seed(0)
    x, s = torch.randn(xs), torch.randn(ss)
    xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yr = _ref(xr, sr)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    xd, sd = x.to(gpu_device).requires_grad_(True), s.to(gpu_device).requires_grad_(True)
    yd = F.complex_join(xd, sd)
    assert torch.equal(yd.cpu(), yr.detach())
    (yd * g.to(gpu_device)).sum().backward()
    assert torch.equal(xd.grad.cpu(), xr.grad)
    assert torch.equal(sd.grad.cpu(), sr.grad)
