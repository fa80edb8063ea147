"""GPU parity of the drop-in constructor variants beyond the BASELINE configs
(VERDICT r4 item 1), against goldens generated from the reference itself
(tests/golden/gen_golden.py variant_cases):
- DCCRN masks 'R' and 'C' (_2008_00264_dccrn.py:127-132, 188-193), DCCRN-CL with
  bidirectional=True (:124, 143; LSTMBlock :60-64), the real-valued DCCRN
  (is_complex=False: nn.Conv2d / BatchNorm2d / PReLU blocks, nn.LSTM + nn.Linear);
- DCUNet-10, DCUNet-20 and DCUNet-20-large (architectures.py:55-98), the last at the
  reference's own test.py settings (1024 / 256 / 1024, 2 s; test.py:8-19).
These reach kernel paths the BASELINE configs do not: (7, 1) / (1, 7) taps at stride
(1, 1), 45 / 90 / 180-channel layers (C % 8 != 0), a 180-channel last encoder layer,
bidirectional recurrences, plain BatchNorm2d + PReLU.
Bar: the north star's 1e-4 relative L2, train and eval mode. Plus the training
gradients of DCUNet-20 per tensor against an fp64 run of the oracle.
(DCUNet with is_complex=False fails inside the reference itself: its first conv expects
1 input channel but the stacked spectrum has 2, _1903_03107_dcunet.py:104-106,118-122;
sehip raises the same way, test_dcunet_real_raises_like_reference.)"""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2
import paramfill

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _variants():
    from sehip import models as M
    return [
        ("dccrn_r", lambda: M.DCCRN("dccrn-R", 400, 100, 512)),
        ("dccrn_c", lambda: M.DCCRN("dccrn-C", 400, 100, 512)),
        ("dccrn_bi", lambda: M.DCCRN("dccrn-CL", 400, 100, 512, bidirectional=True)),
        ("dccrn_real", lambda: M.DCCRN("dccrn-CL", 400, 100, 512, is_complex=False)),
        ("dcunet10", lambda: M.DCUNet("dcunet10", 512, 128, 512)),
        ("dcunet20", lambda: M.DCUNet("dcunet20", 512, 128, 512)),
        ("dcunet20_large", lambda: M.DCUNet("dcunet20-large", 1024, 256, 1024)),
    ]


NAMES = ["dccrn_r", "dccrn_c", "dccrn_bi", "dccrn_real", "dcunet10", "dcunet20", "dcunet20_large"]


@pytest.mark.parametrize("i", range(len(NAMES)), ids=NAMES)
def test_variant_forward_golden(i, gpu_device):
    name, ctor = _variants()[i]
    g = golden(f"variant_{name}")
    m = paramfill.fill_(ctor(), seed=70 + i).cuda()
    x = torch.from_numpy(g["x"]).cuda()
    with torch.no_grad():
        for mode in ("train", "eval"):
            spec, wav = (m.train() if mode == "train" else m.eval())(x)
            torch.cuda.synchronize()
            es = rel_l2(spec.cpu().numpy(), g[f"spec_{mode}"])
            ew = rel_l2(wav.cpu().numpy(), g[f"wav_{mode}"])
            print(f"{name} {mode}: spec {es:.2e} wav {ew:.2e}")
            assert es < TOL and ew < TOL, (name, mode, es, ew)


def _dcunet20_grads(dev, dtype, sehip=False, perturb=0.0, seed=1234):
    from oracle import models as O, train as OT
    noisy, clean = paramfill.structured_pair(1, 32000, seed=42)
    if sehip:
        from sehip import models as M
        from sehip.losses import SI_SNR_loss as loss_fn, pad_or_truncate_wav as pad
        m = M.DCUNet("dcunet20", 512, 128, 512)
    else:
        loss_fn, pad = OT.si_snr_loss, OT.pad_or_truncate_wav
        m = O.DCUNet("dcunet20", 512, 128, 512)
    m = paramfill.fill_(m, seed=75).to(dev).to(dtype).train()
    # the reference's 'bounded_sigmoid' mask (_1903_03107_dcunet.py:166-168) instead of the
    # default 'bounded_tanh', whose mask_phase / mask_mag (:177) makes the gradient chaotic
    # at random init (the fp32 CPU oracle lands 1.5x its own norm off fp64): the gate then
    # measures the conv / CBN backward of every layer, not the phase term's conditioning
    if sehip:
        m._mask_processing = lambda h, noisy: noisy * torch.sigmoid(h)
    else:
        m._mask = lambda h, noisy: noisy * torch.sigmoid(h)
    x = torch.from_numpy(noisy).to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=torch.float64)).to(dtype)
    c = torch.from_numpy(clean).to(dev).to(dtype)
    _, w = m(x.to(dev))
    loss_fn(pad(w, c), c).backward()
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}


def test_dcunet20_train_grads_vs_fp64(gpu_device):
    """DCUNet-20 training gradients (its (7, 1) / (1, 7) stride-1 first encoder layers and
    the 45 / 90 / 180-channel GEMM shapes, forward, data- and weight-grads) per tensor
    against an fp64 CPU run of the oracle: each within max(3x the largest error of the
    fp32 CPU evaluations (unperturbed, and two 2^-22 input perturbations), 1e-4), and the
    median within 3x the largest median of those evaluations."""
    g64 = _dcunet20_grads("cpu", torch.float64)
    evals = [_dcunet20_grads("cpu", torch.float32)] + \
        [_dcunet20_grads("cpu", torch.float32, perturb=2.0 ** -22, seed=1234 + i) for i in range(2)]
    gh = _dcunet20_grads("cuda", torch.float32, sehip=True)
    assert sorted(gh) == sorted(g64)
    rel = lambda g, n: (g[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30)
    rows = [(rel(gh, n), max(rel(q, n) for q in evals), n) for n in g64]
    bad = [r for r in rows if r[0] > max(3 * r[1], 1e-4)]
    med_h = np.median([r[0] for r in rows])
    med_o = max(np.median([rel(q, n) for n in g64]) for q in evals)
    print(f"dcunet20 grads vs fp64: median hip {med_h:.2e}, fp32 evaluations up to {med_o:.2e}; "
          f"worst {max(rows, key=lambda r: r[0] / max(r[1], 1e-12))}")
    assert not bad, sorted(bad, key=lambda r: -r[0])[:5]
    assert med_h < 3 * med_o, (med_h, med_o)


def test_dcunet_real_raises_like_reference(gpu_device):
    from sehip import models as M
    m = M.DCUNet("dcunet16", 512, 128, 512, is_complex=False).cuda()
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 32000, device="cuda"))


def _dcunet16_tanh_grads(dev, dtype, sehip=False, perturb=0.0, seed=1234):
    """DCUNet-16 with its DEFAULT 'bounded_tanh' mask (_1903_03107_dcunet.py:158-184), the
    training backward of the whole model, fp64 / fp32 on the CPU (oracle) or the HIP path."""
    from oracle import models as O, train as OT
    noisy, clean = paramfill.structured_pair(1, 32000, seed=42)
    if sehip:
        from sehip import models as M
        from sehip.losses import SI_SNR_loss as loss_fn, pad_or_truncate_wav as pad
        m = M.DCUNet("dcunet16", 512, 128, 512)
    else:
        loss_fn, pad = OT.si_snr_loss, OT.pad_or_truncate_wav
        m = O.DCUNet("dcunet16", 512, 128, 512)
    m = paramfill.fill_(m, seed=75).to(dev).to(dtype).train()
    x = torch.from_numpy(noisy).to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=torch.float64)).to(dtype)
    c = torch.from_numpy(clean).to(dev).to(dtype)
    _, w = m(x.to(dev))
    loss_fn(pad(w, c), c).backward()
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}


def test_dcunet16_bounded_tanh_train_grads_vs_fp64(gpu_device):
    """The default mask's training gradients through the whole model.
    At random init this mask's gradient is ill-conditioned (profiles/r6_dcunet_tanh_spread.log,
    tools/dcunet_tanh_spread.py): a 2^-22 relative input perturbation moves the fp64 gradient by
    5.7e-2 / 7.3e-2 median per tensor, and the fp32 CPU oracle lands 3.6e-1 off fp64. The gate
    is therefore anchored on those fp32 evaluations (as DCCRN's and DCUNet-20's): each tensor
    within 3x the largest fp32-evaluation error of fp64, and the median within 3x the largest
    median. (The well-conditioned 'bounded_sigmoid' form is gated tightly by
    test_dcunet20_train_grads_vs_fp64, the op by tests/test_gpu_polar_mask.py.)"""
    g64 = _dcunet16_tanh_grads("cpu", torch.float64)
    evals = [_dcunet16_tanh_grads("cpu", torch.float32)] + \
        [_dcunet16_tanh_grads("cpu", torch.float32, perturb=2.0 ** -22, seed=1234 + i) for i in range(2)]
    gh = _dcunet16_tanh_grads("cuda", torch.float32, sehip=True)
    assert sorted(gh) == sorted(g64)
    assert all(torch.isfinite(g).all() for g in gh.values())
    rel = lambda g, n: (g[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30)
    rows = [(rel(gh, n), max(rel(q, n) for q in evals), n) for n in g64]
    bad = [r for r in rows if r[0] > max(3 * r[1], 1e-4)]
    med_h = np.median([r[0] for r in rows])
    med_o = max(np.median([rel(q, n) for n in g64]) for q in evals)
    print(f"dcunet16 bounded_tanh grads vs fp64: median hip {med_h:.2e}, fp32 evaluations up to {med_o:.2e}")
    assert not bad, sorted(bad, key=lambda r: -r[0])[:5]
    assert med_h < 3 * med_o, (med_h, med_o)
