"""ComplexBatchNorm moments written by the conv's forward GEMM epilogue
(se_conv2d_desc.moments, ABI 5) and consumed by se_cbn_fwd_moments /
se_cbn_head_fwd_moments instead of the CBN's own pass over y (the reference
computes them inside ComplexBatchNorm2d.forward, complex_nn.py:235-260).

* The moment rows, summed over their M-tiles, equal fp64 sums of the conv output
  computed by torch (same fp32 values; only the fp64 summation order differs), and
  the extrema are exact.
* A CBN forward from those rows equals the CBN's own pass (outputs, running
  statistics, gradients).
* The FRCRN train step with the epilogue moments (default) matches
  SEHIP_CONV_MOMENTS=0, and every moment row written is consumed.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _moments_on(monkeypatch):
    monkeypatch.setenv("SEHIP_CONV_MOMENTS", "1")   # opt-in path (off by default)

GEOMS = [   # (x shape, out channels, kernel, stride, padding, transposed)
    ((2, 128, 33, 37), 128, (5, 2), (2, 1), (2, 0), False),    # FRCRN encoder conv: 4-wave tiles, M tail
    ((2, 128, 17, 37), 128, (5, 2), (2, 1), (2, 0), True),     # decoder convT: two stride-phase classes
    ((2, 96, 12, 50), 256, (3, 3), (1, 1), (1, 1), False),     # N = 256: 8-wave tiles
    ((1, 128, 5, 7), 130, (3, 3), (1, 1), (1, 1), False),      # N = 130, 35 positions (one partial tile)
]


def _check_rows(y, buf, rows, cout):
    Cc = cout // 2
    part = buf[:Cc * rows * 40].view(torch.float64).view(Cc, rows, 5)
    ext = buf[Cc * rows * 40:Cc * rows * 56].view(torch.float32).view(Cc, rows, 4)
    yd = y.double()
    yr, yi = yd[:, :Cc], yd[:, Cc:]
    ref = torch.stack([yr.sum((0, 2, 3)), yi.sum((0, 2, 3)), (yr * yr).sum((0, 2, 3)),
                       (yr * yi).sum((0, 2, 3)), (yi * yi).sum((0, 2, 3))], 1)
    scale = torch.stack([yr.abs().sum((0, 2, 3)), yi.abs().sum((0, 2, 3)), (yr * yr).sum((0, 2, 3)),
                         (yr * yi).abs().sum((0, 2, 3)), (yi * yi).sum((0, 2, 3))], 1)
    got = part.sum(1)
    assert ((got - ref).abs() <= 1e-12 * scale + 1e-300).all(), (got - ref).abs().max().item()
    f = y.float()
    fr, fi = f[:, :Cc], f[:, Cc:]
    ref_e = torch.stack([fr.amax((0, 2, 3)), -fr.amin((0, 2, 3)), fi.amax((0, 2, 3)), -fi.amin((0, 2, 3))], 1)
    assert torch.equal(ext.amax(1), ref_e)


@pytest.mark.parametrize("geom", GEOMS)
def test_conv_moment_rows_match_fp64(gpu_device, geom):
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math("f16x3")
    try:
        torch.manual_seed(0)
        xs, cout, k, st, pad, tr = geom
        cin = xs[1]
        wshape = (cin // 2, cout // 2) + k if tr else (cout // 2, cin // 2) + k
        x = torch.randn(xs, device=gpu_device) + 0.3
        wr, wi = torch.randn(wshape, device=gpu_device) * 0.05, torch.randn(wshape, device=gpu_device) * 0.05
        n0 = F.MOMENT_CALLS[0]
        with F.emit_moments(True):
            y = F.conv2d(x, wr, wi, out_channels=cout, kernel=k, stride=st, padding=pad, transposed=tr)
        with torch.no_grad():
            y_ref = F.conv2d(x, wr, wi, out_channels=cout, kernel=k, stride=st, padding=pad, transposed=tr)
        assert torch.equal(y, y_ref)    # the epilogue only adds the moment rows
        assert F.MOMENT_CALLS[0] == n0 + 1
        e = F.moments_take(y)
        assert e is not None
        torch.cuda.synchronize()
        _check_rows(y, e[0], e[1], cout)
    finally:
        F.set_conv_math(prev)


def test_joined_conv_moment_rows_match_fp64(gpu_device):
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math("f16x3")
    try:
        torch.manual_seed(2)
        x, s = torch.randn(2, 128, 8, 38, device=gpu_device), torch.randn(2, 128, 9, 37, device=gpu_device)
        wr = torch.randn(128, 64, 5, 2, device=gpu_device) * 0.05
        wi = torch.randn(128, 64, 5, 2, device=gpu_device) * 0.05
        with F.emit_moments(True):
            y = F.conv2d_joined(x, s, wr, wi, out_channels=128, kernel=(5, 2), stride=(2, 1), transposed=True)
        e = F.moments_take(y)
        assert e is not None
        torch.cuda.synchronize()
        _check_rows(y, e[0], e[1], 128)
    finally:
        F.set_conv_math(prev)


def test_unsupported_shape_runs_without_moments(gpu_device):
    """N > 256 output channels: no epilogue moments; the conv result is unchanged and the
    CBN later runs its own pass."""
    from sehip import functional as F
    torch.manual_seed(3)
    x = torch.randn(1, 64, 9, 20, device=gpu_device)
    wr, wi = torch.randn(160, 32, 3, 3, device=gpu_device) * 0.05, torch.randn(160, 32, 3, 3, device=gpu_device) * 0.05
    with F.emit_moments(True):
        y = F.conv2d(x, wr, wi, out_channels=320, kernel=(3, 3), padding=(1, 1))
    assert F.moments_take(y) is None
    y_ref = F.conv2d(x, wr, wi, out_channels=320, kernel=(3, 3), padding=(1, 1))
    assert torch.equal(y, y_ref)


@pytest.mark.parametrize("act", [0, 1])
def test_cbn_forward_from_conv_moments(gpu_device, act):
    """se_cbn_fwd_moments against se_cbn_fwd on the same conv output: outputs, running
    statistics and input / parameter gradients (fp64 sums in another order only)."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d
    torch.manual_seed(4)
    x = torch.randn(2, 128, 33, 37, device=gpu_device) * 2 + 0.5
    wr = torch.randn(64, 64, 5, 2, device=gpu_device) * 0.05
    wi = torch.randn(64, 64, 5, 2, device=gpu_device) * 0.05
    kw = dict(out_channels=128, kernel=(5, 2), stride=(2, 1), padding=(2, 0))
    outs = []
    bn0 = ComplexBatchNorm2d(128).to(gpu_device).train()   # Wri is drawn at random: one state for both runs
    with torch.no_grad():
        bn0.Wrr.add_(0.3)
        bn0.Br.add_(0.1)
    for emit in (True, False):
        bn = ComplexBatchNorm2d(128).to(gpu_device).train()
        bn.load_state_dict(bn0.state_dict())
        xa = x.clone().requires_grad_(True)
        n1 = F.MOMENT_CALLS[1]
        with F.emit_moments(emit):
            y = F.conv2d(xa, wr, wi, **kw)
        z = bn.forward_act(y, act, 0.2)
        assert F.MOMENT_CALLS[1] == n1 + int(emit)
        g = torch.randn(z.shape, device=gpu_device, generator=torch.Generator(gpu_device).manual_seed(1))
        z.backward(g)
        torch.cuda.synchronize()
        outs.append((z.detach(), xa.grad, bn.Wrr.grad, bn.Br.grad, bn.RMr.clone(), bn.RVrr.clone(),
                     bn.RVri.clone()))
    for name, a, b in zip(("z", "dx", "dWrr", "dBr", "RMr", "RVrr", "RVri"), *outs):
        err = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert err <= 1e-6, (name, err)


def test_frcrn_step_with_conv_moments(gpu_device, monkeypatch):
    """FRCRN forward + backward with the epilogue moments (SEHIP_CONV_MOMENTS=1) against
    SEHIP_CONV_MOMENTS=0: every CBN fed by a split-fp16 conv (encoder blocks 1-5, the
    decoder blocks and the fused head) reads moment rows, every row written is read,
    and the output and gradients agree."""
    import paramfill
    from sehip import functional as F
    from sehip.losses import SI_SNR_loss
    from sehip.models import FRCRN

    def run():
        m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
        noisy, clean = (torch.from_numpy(t).cuda() for t in paramfill.structured_pair(2, 16000, seed=60))
        _, wav = m(noisy)
        SI_SNR_loss(wav, clean).backward()
        torch.cuda.synchronize()
        return wav.detach(), {n: p.grad.detach() for n, p in m.named_parameters()}

    monkeypatch.setenv("SEHIP_CONV_MOMENTS", "0")
    c0 = list(F.MOMENT_CALLS)
    w0, g0 = run()
    assert F.MOMENT_CALLS == c0
    monkeypatch.setenv("SEHIP_CONV_MOMENTS", "1")
    w1, g1 = run()
    made, used = F.MOMENT_CALLS[0] - c0[0], F.MOMENT_CALLS[1] - c0[1]
    assert made == used and made >= 10, (made, used)
    assert ((w1 - w0).norm() / w0.norm()).item() <= 1e-5
    errs = sorted(((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-30)).item() for n in g0)
    assert errs[len(errs) // 2] <= 1e-5 and errs[-1] <= 1e-3, (errs[len(errs) // 2], errs[-1])
