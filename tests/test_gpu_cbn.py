"""GPU parity: ComplexBatchNorm2d kernels (csrc/cbn.hip) vs reference goldens:
train-mode forward, running-stat update, backward (dx and all 5 affine
params), eval-mode forward/backward; plus fused LeakyReLU vs oracle."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2
import paramfill

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,C,seed", [("c5", 10, 0), ("c1", 2, 1)])
def test_cbn_golden(name, C, seed, gpu_device):
    from sehip.complex_nn import ComplexBatchNorm2d
    g = golden("cbn")
    m = paramfill.fill_(ComplexBatchNorm2d(C), seed=seed).cuda().train()
    x = torch.from_numpy(g[f"{name}_x"]).cuda().requires_grad_(True)
    y = m(x)
    assert rel_l2(y.detach().cpu().numpy(), g[f"{name}_y"]) < 1e-5
    (y * torch.from_numpy(g[f"{name}_gy"]).cuda()).sum().backward()
    assert rel_l2(x.grad.cpu().numpy(), g[f"{name}_dx"]) < 1e-5
    dp = torch.cat([m.Wrr.grad, m.Wri.grad, m.Wii.grad, m.Br.grad, m.Bi.grad]).cpu().numpy()
    assert rel_l2(dp, g[f"{name}_dparams"]) < 1e-5
    run = torch.cat([m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii]).cpu().numpy()
    np.testing.assert_allclose(run, g[f"{name}_run1"], rtol=1e-5, atol=1e-6)
    assert int(m.num_batches_tracked) == 1
    m2 = paramfill.fill_(ComplexBatchNorm2d(C), seed=seed).cuda().eval()
    xe = torch.from_numpy(g[f"{name}_x"]).cuda().requires_grad_(True)
    ye = m2(xe)
    assert rel_l2(ye.detach().cpu().numpy(), g[f"{name}_yeval"]) < 1e-5
    (ye * torch.from_numpy(g[f"{name}_gy"]).cuda()).sum().backward()
    assert rel_l2(xe.grad.cpu().numpy(), g[f"{name}_dxeval"]) < 1e-5
    dpe = torch.cat([m2.Wrr.grad, m2.Wri.grad, m2.Wii.grad, m2.Br.grad, m2.Bi.grad]).cpu().numpy()
    assert rel_l2(dpe, g[f"{name}_dparamseval"]) < 1e-5


def test_cbn_leaky_fused_vs_oracle(gpu_device):
    """FRCRN-shaped CBN(128) + LeakyReLU(0.2), fused in one kernel, vs oracle."""
    from sehip.complex_nn import ComplexBatchNorm2d, norm_act
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(3, 128, 17, 41, generator=gen) * 2 + 0.5
    gy = torch.randn(x.shape, generator=gen)
    mo = paramfill.fill_(OCBN(128), seed=2).train()
    xo = x.clone().requires_grad_(True)
    yo = torch.nn.functional.leaky_relu(mo(xo), 0.2)
    yo.backward(gy)
    m = paramfill.fill_(ComplexBatchNorm2d(128), seed=2).cuda().train()
    xg = x.cuda().requires_grad_(True)
    y = norm_act(m, torch.nn.LeakyReLU(0.2), xg)
    y.backward(gy.cuda())
    assert rel_l2(y.detach().cpu().numpy(), yo.detach().numpy()) < 1e-5
    assert rel_l2(xg.grad.cpu().numpy(), xo.grad.numpy()) < 1e-4
    for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert rel_l2(getattr(m, n).grad.cpu().numpy(), getattr(mo, n).grad.numpy()) < 1e-4, n
    for n in ("RMr", "RMi", "RVrr", "RVri", "RVii"):
        np.testing.assert_allclose(getattr(m, n).cpu().numpy(), getattr(mo, n).detach().numpy(),
                                   rtol=1e-5, atol=1e-6)


def test_cbn_whitening_full_size(gpu_device):
    """Known answer: with W = I, B = 0 the train-mode output is
    whitened — zero mean, identity covariance — at an FRCRN activation size."""
    from sehip.complex_nn import ComplexBatchNorm2d
    m = ComplexBatchNorm2d(128).cuda().train()
    with torch.no_grad():
        m.Wri.zero_()
    x = torch.randn(8, 128, 77, 403, device="cuda") * 3 + 1.5
    x[:, 64:] += 0.7 * x[:, :64]          # correlate real / imag
    y = m(x).double()
    yr, yi = y[:, :64], y[:, 64:]
    assert yr.mean(dim=(0, 2, 3)).abs().max() < 1e-5
    assert (yr.pow(2).mean(dim=(0, 2, 3)) - 1).abs().max() < 1e-3
    assert (yi.pow(2).mean(dim=(0, 2, 3)) - 1).abs().max() < 1e-3
    assert (yr * yi).mean(dim=(0, 2, 3)).abs().max() < 1e-3


@pytest.mark.parametrize("act", [0, 1, 2])
def test_cbn_amax_bounds(act, gpu_device):
    """The SE_MATH_F16X3 scale sources se_cbn_fwd / se_cbn_bwd emit with no extra
    pass: an upper bound of max |y| and of max |dx| (never below the true
    maximum, at most a small factor above it)."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d
    seen = {}

    class Probe(torch.autograd.Function):   # sees dx with the address the CBN backward registered
        @staticmethod
        def forward(ctx, t):
            return t.view(t.shape)

        @staticmethod
        def backward(ctx, g):
            seen["dx"], seen["dx_amax"] = g.clone(), F.amax_get(g)
            return g

    m = paramfill.fill_(ComplexBatchNorm2d(128), seed=3).cuda().train()
    gen = torch.Generator(device=gpu_device).manual_seed(9)
    x = (torch.randn(4, 128, 37, 50, device=gpu_device, generator=gen) * 3 + 0.5).requires_grad_(True)
    y = m.forward_act(Probe.apply(x), act, 0.2)
    ya = F.amax_get(y)
    assert ya is not None
    true_y = y.detach().abs().max().item()
    assert true_y <= ya.item() <= 4 * true_y, (true_y, ya.item())
    gy = torch.randn(y.shape, device=gpu_device, generator=gen) * 1e-7
    y.backward(gy)
    assert seen["dx_amax"] is not None
    true_dx = seen["dx"].abs().max().item()
    assert true_dx <= seen["dx_amax"].item() <= 16 * true_dx, (true_dx, seen["dx_amax"].item())


@pytest.mark.parametrize("used", ["both", "first", "second"])
def test_cbn_fork_sums_both_gradients(used, gpu_device):
    """fork=True (FRCRN encoder outputs: next conv + decoder skip) sums the two output
    gradients inside se_cbn_bwd2; bit-identical to autograd's add followed by se_cbn_bwd,
    and either consumer alone (the other gradient absent) matches the plain backward."""
    from sehip.complex_nn import ComplexBatchNorm2d, norm_act
    gen = torch.Generator().manual_seed(11)
    x = (torch.randn(4, 128, 13, 37, generator=gen) * 1.5 + 0.3).cuda()
    g1 = torch.randn(x.shape, generator=gen).cuda()
    g2 = torch.randn(x.shape, generator=gen).cuda()
    grads = {"both": (g1, g2), "first": (g1, None), "second": (None, g2)}[used]
    act = torch.nn.LeakyReLU(0.2)

    m0 = paramfill.fill_(ComplexBatchNorm2d(128), seed=4).cuda().train()
    x0 = x.clone().requires_grad_(True)
    y0 = norm_act(m0, act, x0)
    y0.backward(sum(g for g in grads if g is not None))

    m1 = paramfill.fill_(ComplexBatchNorm2d(128), seed=4).cuda().train()
    x1 = x.clone().requires_grad_(True)
    ya, yb = norm_act(m1, act, x1, fork=True)
    assert yb.data_ptr() == ya.data_ptr() and torch.equal(ya, y0)
    outs = [(t, g) for t, g in zip((ya, yb), grads) if g is not None]
    torch.autograd.backward([t for t, _ in outs], [g for _, g in outs])
    assert torch.equal(x1.grad, x0.grad)
    for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert torch.equal(getattr(m1, n).grad, getattr(m0, n).grad), n
