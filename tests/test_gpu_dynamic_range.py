"""Dynamic range of the f16x3 conv arithmetic (the headline's default MFMA form).

f16x3 scales each GEMM operand by a power of two before splitting it into
hi + lo fp16 halves (functional.py). Real training batches mix
utterances across a wide range of levels, and the reference mixer draws SNRs
in [-20, 20] dB (/root/reference/mix_audio.py:95-100). These tests hold the
arithmetic to the north-star bar on such batches, per utterance:

* FRCRN B = 16 x 4 s, train mode (frcrn.py:119-155): per-utterance gains from
  1 down to 2^-16 (96 dB), one utterance with 1 s of digital silence, one
  mixed at -20 dB SNR. Each utterance's spectrum and waveform within 1e-4
  rel-L2 of the CPU oracle (the reference restated, pinned by the goldens).
* The train step's gradients at B = 4 on the same kind of batch, against an
  fp64 oracle run with the per-tensor gate of test_frcrn_train_step_golden.
* One conv pass at a time at FRCRN layer shapes, with operands whose batch
  items sit 2^0 .. 2^-24 apart: the error of every batch item's slice against
  fp64, next to the exact-fp32 MFMA path's.
"""
import numpy as np
import pytest
import torch

from conftest import rel_l2
import paramfill

pytestmark = pytest.mark.gpu

TOL = 1e-4   # north_star: "within 1e-4 rel fp32", per utterance


def level_spread_batch(batch, length, seed, min_log2=-16.0):
    """Structured noisy/clean pairs (paramfill.structured_pair) at per-utterance
    gains 2^0 .. 2^min_log2 (log-spaced). Utterance 1 carries 1 s of digital
    silence (both signals exactly 0) and utterance 2 is re-mixed at -20 dB SNR
    (the reference mixer's lower bound, mix_audio.py:98)."""
    noisy, clean = paramfill.structured_pair(batch, length, seed=seed)
    noisy, clean = noisy.astype(np.float64), clean.astype(np.float64)
    rs = np.random.RandomState(seed + 1)
    if batch > 2:
        noise = rs.standard_normal(length)
        pc, pn = np.mean(clean[2] ** 2), np.mean(noise ** 2)
        noisy[2] = clean[2] + noise * np.sqrt(pc / (pn * 10 ** (-20 / 10)))
    if batch > 1:
        a = min(16000, length // 4)
        noisy[1, a:a + 16000] = 0.0
        clean[1, a:a + 16000] = 0.0
    gains = 2.0 ** np.linspace(0.0, min_log2, batch)
    gains = gains[rs.permutation(batch)]     # quiet and loud items interleaved in the batch
    noisy *= gains[:, None]
    clean *= gains[:, None]
    return noisy.astype(np.float32), clean.astype(np.float32), gains


@pytest.mark.parametrize("min_log2", [-16.0, -24.0])
def test_frcrn_b16_level_spread_per_utterance_vs_oracle(min_log2, gpu_device):
    from sehip import functional as F
    from sehip import models as M
    from oracle import models as O
    assert F.get_conv_math() == "f16x3"      # the headline's arithmetic
    noisy, _, gains = level_spread_batch(16, 64000, seed=41, min_log2=min_log2)
    mo = paramfill.fill_(O.FRCRN(), seed=43).train()
    m = paramfill.fill_(M.FRCRN(), seed=43).cuda().train()
    with torch.no_grad():
        so, wo = mo(torch.from_numpy(noisy))
        s, w = m(torch.from_numpy(noisy).cuda())
    s, w = s.cpu().numpy(), w.cpu().numpy()
    worst = 0.0
    for b in range(16):
        es, ew = rel_l2(s[b], so[b].numpy()), rel_l2(w[b], wo[b].numpy())
        print(f"utt {b:2d} gain 2^{np.log2(gains[b]):6.2f}: spec {es:.2e} wav {ew:.2e}")
        worst = max(worst, es, ew)
        assert es < TOL and ew < TOL, (b, gains[b], es, ew)
    print(f"worst per-utterance rel-L2 {worst:.2e}")


def _oracle_grads(noisy, clean, dtype, perturb=0.0, seed=1234):
    from oracle import models as O, train as OT
    x, c = torch.from_numpy(noisy).to(dtype), torch.from_numpy(clean).to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=dtype))
    m = paramfill.fill_(O.FRCRN(), seed=47).to(dtype).train()
    if perturb:   # the weights re-rounded too: a stand-in for the rounding inside every layer
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(1 + perturb * torch.randn(p.shape, generator=gen, dtype=dtype))
    _, w = m(x[:, None])
    OT.si_snr_loss(OT.pad_or_truncate_wav(w, c), c).backward()
    return {n: p.grad.double() for n, p in m.named_parameters()}


@pytest.mark.timeout(400)
def test_frcrn_level_spread_train_step_grads_vs_fp64(gpu_device):
    """B = 4 x 4 s with gains 1, 2^-5.3, 2^-10.7, 2^-16 (the silence and -20 dB
    items included): SI-SNR makes each utterance's gradient scale as 1/level,
    so the backward's operands spread as widely as the forward's. Gate as
    test_frcrn_train_step_golden: every parameter gradient within
    max(3x the fp32 oracle's error, 3x its 2-ulp sensitivity, 1e-4) of fp64, the
    median within 3x the fp32 oracle's median. The sensitivity is the largest move
    of the fp32 oracle over four perturbations of the input and the weights at
    2^-20 relative: the size of the HIP path's own deviation from fp64 (per conv
    4.0e-7 f16x3 / 6.4e-7 exact fp32 MFMA; at the model output 1-2.6e-6 per
    utterance, test_frcrn_b16_level_spread_per_utterance_vs_oracle). For a
    well-conditioned gradient that move is ~1e-6, under the 1e-4 floor, so the
    gate only widens for the chaotic ones: a few CCBAM spatial-attention gradients route
    through channel max-pools whose argmax flips under any re-rounding. Measured on
    the CPU oracle for skip layer 3's spatial...norm.Wri (fp32 vs fp64: 6.2e-3):
    perturbations at 2^-22 move it up to 1.0e-2, at 2^-20 up to 5.7e-2, at 2^-18
    up to 1.1 (a chaotic gradient, not a precision signal)."""
    from sehip import models as M
    from sehip.losses import SI_SNR_loss, pad_or_truncate_wav
    noisy, clean, gains = level_spread_batch(4, 64000, seed=51)
    m = paramfill.fill_(M.FRCRN(), seed=47).cuda().train()
    c = torch.from_numpy(clean).cuda()
    _, wav = m(torch.from_numpy(noisy).cuda()[:, None])
    SI_SNR_loss(pad_or_truncate_wav(wav, c), c).backward()
    torch.cuda.synchronize()
    g64 = _oracle_grads(noisy, clean, torch.float64)
    g32 = _oracle_grads(noisy, clean, torch.float32)
    g32ps = [_oracle_grads(noisy, clean, torch.float32, perturb=2.0 ** -20, seed=1234 + i) for i in range(4)]
    errs = []
    for n, p in m.named_parameters():
        d = g64[n].norm().item() + 1e-300
        errs.append(((p.grad.double().cpu() - g64[n]).norm().item() / d,
                     (g32[n] - g64[n]).norm().item() / d,
                     max((q[n] - g32[n]).norm().item() for q in g32ps) / d, n))
    med_hip, med_32 = np.median([e[0] for e in errs]), np.median([e[1] for e in errs])
    worst = max(errs, key=lambda e: e[0] / max(e[1], e[2], 1e-12))
    print(f"gains {np.log2(gains).round(2)}: median grad err vs fp64 hip {med_hip:.2e} cpu-fp32 {med_32:.2e}; "
          f"worst ratio {worst}")
    bad = [e for e in errs if e[0] > max(3 * e[1], 3 * e[2], 1e-4)]
    assert not bad, bad[:5]
    assert med_hip < 3 * med_32, (med_hip, med_32)


# (name, transposed, Cin, Cout, x shape, stride): FRCRN encoder / decoder layer shapes
LAYERS = [
    ("enc1", False, 128, 128, (4, 128, 77, 41), (2, 1)),
    ("dec5", True, 256, 128, (4, 256, 77, 40), (2, 1)),
]
ITEM_LOG2 = (0.0, -8.0, -16.0, -24.0)


def _conv_case(tr, cin, cout, shape, stride, x_gain, gy_gain):
    from oracle import complex_nn as O_cnn
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, (5, 2), stride=stride, bias=False), seed=7).double()
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(*shape, generator=gen, dtype=torch.float64) * torch.tensor(x_gain)[:, None, None, None]
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    gy = torch.randn(yo.shape, generator=gen, dtype=torch.float64) * torch.tensor(gy_gain)[:, None, None, None]
    yo.backward(gy)
    return m, x, gy, dict(y=yo.detach(), dx=xo.grad, dwr=m.real_conv.weight.grad, dwi=m.imag_conv.weight.grad)


def _hip_conv(m, x, gy, tr, stride, math):
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        wr = m.real_conv.weight.detach().float().cuda().requires_grad_(True)
        wi = m.imag_conv.weight.detach().float().cuda().requires_grad_(True)
        xg = x.float().cuda().requires_grad_(True)
        y = F.conv2d(xg, wr, wi, out_channels=2 * m.real_conv.out_channels, kernel=(5, 2), stride=stride,
                     transposed=tr)
        y.backward(gy.float().cuda())
        torch.cuda.synchronize()
        return dict(y=y.detach().cpu(), dx=xg.grad.cpu(), dwr=wr.grad.cpu(), dwi=wi.grad.cpu())
    finally:
        F.set_conv_math(prev)


def _f16x3_bound(e32, level_log2):
    """The per-tensor-scaled split's error at data 2^level_log2 below the operand's
    max: fp32-class (<= 1.25x the exact path) while the lo half stays normal, i.e.
    down to ~2^-17 of the max; below that the absolute error floor ~2^-38 max of
    fp16 subnormals, measured 2.3 x 2^(L - 38) relative at level 2^-L; bound 4x."""
    return max(1.25 * e32, 2e-7, 4.0 * 2.0 ** (-level_log2 - 38))


@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", LAYERS)
def test_f16x3_per_item_levels_vs_fp64(name, tr, cin, cout, shape, stride, gpu_device):
    """The raw arithmetic (no model-level mitigation): batch items of one operand
    2^0, 2^-8, 2^-16, 2^-24 apart (x and dy in opposite orders). Per item, y and dx
    against fp64 within _f16x3_bound of the item's level (x's for y, dy's for dx);
    the weight gradient, a sum over all items, within the bound of the deepest."""
    x_gain = [2.0 ** v for v in ITEM_LOG2]
    gy_gain = [2.0 ** v for v in ITEM_LOG2[::-1]]
    m, x, gy, ref = _conv_case(tr, cin, cout, shape, stride, x_gain, gy_gain)
    e32 = _hip_conv(m, x, gy, tr, stride, "f32")
    e16 = _hip_conv(m, x, gy, tr, stride, "f16x3")
    for k, r in ref.items():
        items = range(r.shape[0]) if k in ("y", "dx") else [None]
        for b in items:
            sl = (lambda t: t[b]) if b is not None else (lambda t: t)
            lvl = {"y": ITEM_LOG2[b] if b is not None else 0, "dx": ITEM_LOG2[::-1][b] if b is not None else 0}
            level = lvl.get(k, min(ITEM_LOG2))
            a32 = rel_l2(sl(e32[k]).numpy(), sl(r).numpy())
            a16 = rel_l2(sl(e16[k]).numpy(), sl(r).numpy())
            print(f"{name} {k} item {b} (level 2^{level:g}): f32 {a32:.2e} f16x3 {a16:.2e} "
                  f"bound {_f16x3_bound(a32, level):.1e}")
            assert a16 <= _f16x3_bound(a32, level), (name, k, b, a16, a32)


REGION_LOG2 = (0.0, -10.0, -20.0, -30.0)


@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", LAYERS[:1])
def test_f16x3_mixed_magnitude_regions_vs_fp64(name, tr, cin, cout, shape, stride, gpu_device):
    """Inside ONE batch item, blocks of frequency rows of x scaled by 2^0, 2^-10,
    2^-20, 2^-30 (quiet time-frequency regions next to loud ones), dy likewise in
    the opposite order: each output region against fp64 within _f16x3_bound of
    its level (the advisor's mixed-magnitude case; the raw arithmetic)."""
    m, x, gy, ref = _conv_case(tr, cin, cout, shape, stride, [1.0] * shape[0], [1.0] * shape[0])
    H = x.shape[2]
    xs = torch.ones(H, dtype=torch.float64)
    for i, v in enumerate(REGION_LOG2):
        xs[i * H // 4:(i + 1) * H // 4] = 2.0 ** v
    x = x * xs[None, None, :, None]
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    Hy = yo.shape[2]
    gs = torch.ones(Hy, dtype=torch.float64)
    for i, v in enumerate(REGION_LOG2[::-1]):
        gs[i * Hy // 4:(i + 1) * Hy // 4] = 2.0 ** v
    gy = torch.randn(yo.shape, generator=torch.Generator().manual_seed(9), dtype=torch.float64) * gs[None, None, :, None]
    m.zero_grad()
    yo.backward(gy)
    ref = dict(y=yo.detach(), dx=xo.grad)
    e32 = _hip_conv(m, x, gy, tr, stride, "f32")
    e16 = _hip_conv(m, x, gy, tr, stride, "f16x3")
    for k, r in ref.items():
        R = r.shape[2]
        for i in range(4):
            sl = slice(i * R // 4 + 3, (i + 1) * R // 4 - 3)   # away from the region borders
            level = REGION_LOG2[i] if k == "y" else REGION_LOG2[::-1][i]
            a32 = rel_l2(e32[k][:, :, sl].numpy(), r[:, :, sl].numpy())
            a16 = rel_l2(e16[k][:, :, sl].numpy(), r[:, :, sl].numpy())
            print(f"{name} {k} region {i} (level 2^{level:g}): f32 {a32:.2e} f16x3 {a16:.2e}")
            assert a16 <= _f16x3_bound(a32, level), (name, k, i, a16, a32)


def test_first_conv_runs_exact_fp32(gpu_device):
    """Every model marks its first (data-fed) conv: where the conv math is f16x3 its
    passes run the exact fp32 MFMA (the spectrum's level spread never meets the
    per-tensor scale); every later conv keeps f16x3."""
    from sehip import functional as F
    from sehip import models as M
    timer = F.OpTimer()
    m = paramfill.fill_(M.FRCRN(), seed=3).cuda().train()
    noisy, clean = paramfill.structured_pair(2, 16000, seed=2)
    F.set_op_timer(timer)
    try:
        _, wav = m(torch.from_numpy(noisy).cuda())
        (wav * torch.from_numpy(clean).cuda()).sum().backward()
    finally:
        F.set_op_timer(None)
    tags = [r[0] for r in timer.records if r[0].startswith("conv_")]
    # the first conv's weight-grad: exact fp32 products inside the fused first block's CBN
    # backward (se_cbn_bwd_first_conv), or the fp32 weight-grad GEMM (SEHIP_FIRST_FUSED=0)
    fused = sum(r[0] == "cbn_bwd_first_conv" for r in timer.records)
    assert tags.count("conv_fwd_f32") == 1 and tags.count("conv_wgrad_f32") + fused == 1, tags
    assert tags.count("conv_fwd_f16x3") == 5 and "conv_data_f32" not in tags, tags
