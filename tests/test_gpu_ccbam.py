"""Fused CCBAM (csrc/ccbam.hip + the sub-modules' HIP conv/CBN) against the
oracle's restatement of models/modules/ccbam.py on the CPU (fp32):
forward output, input gradient, every parameter gradient and the spatial
CBN's running statistics. Tolerance: rel-L2 <= 1e-5 forward, <= 1e-4 for
gradients (reduction order only; the gate's sigmoid/CBN chain is smooth).

Ties: the fused kernels send max-pool gradients to the first maximal index
(AdaptiveMaxPool2d, torch.max(dim)); continuous random inputs have no ties,
so the comparison is exact in structure."""
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


@pytest.mark.parametrize("B,C,H,W", [(2, 32, 9, 13), (3, 128, 7, 403), (2, 128, 2, 403), (1, 4, 5, 5)])
def test_ccbam_matches_oracle(gpu_device, B, C, H, W):
    from oracle.ccbam import CCBAM as OCCBAM
    from sehip.ccbam import CCBAM
    torch.manual_seed(B * 1000 + C + H)
    ref = OCCBAM(C).train()
    mod = CCBAM(C).train()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(B, C, H, W)
    g = torch.randn(B, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    (yr * g).sum().backward()
    mod = mod.to(gpu_device)
    xd = x.to(gpu_device).requires_grad_(True)
    yd = mod(xd)
    assert _rel(yd, yr) < 1e-5
    (yd * g.to(gpu_device)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-4
    rp = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert p.grad is not None, n
        assert _rel(p.grad, rp[n].grad) < 1e-4, (n, _rel(p.grad, rp[n].grad))
    rb = dict(ref.named_buffers())
    for n, b in mod.named_buffers():
        if b.dtype.is_floating_point:
            assert _rel(b, rb[n]) < 1e-5, n


def test_ccbam_eval_and_no_grad(gpu_device):
    from oracle.ccbam import CCBAM as OCCBAM
    from sehip.ccbam import CCBAM
    torch.manual_seed(5)
    ref = OCCBAM(32).eval()
    mod = CCBAM(32).eval()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 32, 6, 20)
    with torch.no_grad():
        yd = mod.to(gpu_device)(x.to(gpu_device))
    assert _rel(yd, ref(x)) < 1e-5


def test_ccbam_fused_matches_unfused_on_gpu(gpu_device):
    """The fused path against the module's own op-by-op formulation on the GPU
    at an FRCRN skip shape (B=8 of the B=64 decoder input, F=37)."""
    from sehip.ccbam import CCBAM
    torch.manual_seed(7)
    mod = CCBAM(128).to(gpu_device).train()
    x = torch.randn(8, 128, 37, 403, device=gpu_device)
    g = torch.randn_like(x)
    x1 = x.clone().requires_grad_(True)
    y1 = mod.forward_unfused(x1)
    (y1 * g).sum().backward()
    g1 = {n: p.grad.clone() for n, p in mod.named_parameters()}
    mod.zero_grad(set_to_none=True)
    x2 = x.clone().requires_grad_(True)
    y2 = mod(x2)
    (y2 * g).sum().backward()
    assert _rel(y2, y1) < 1e-5
    assert _rel(x2.grad, x1.grad) < 1e-4
    for n, p in mod.named_parameters():
        assert _rel(p.grad, g1[n]) < 1e-4, n
