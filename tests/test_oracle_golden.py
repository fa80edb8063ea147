"""Pin the oracle restatement against fixtures generated from the reference.

CPU only. Tolerances: the oracle runs the same fp32 ATen ops as the
reference in a different order (e.g. one mean over (0,2,3) instead of three
sequential means), so agreement is ~1e-6 relative.
"""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2
import paramfill
from oracle import stft as O_stft, complex_nn as O_cnn, ccbam as O_ccbam, models as O_models, train as O_train

torch.set_num_threads(4)

STFT_CONFIGS = [(320, 160, 640), (400, 100, 512), (512, 128, 512),
                (320, 160, 512), (320, 160, 320), (1024, 256, 1024)]


@pytest.mark.parametrize("cfg", STFT_CONFIGS)
def test_stft_basis_and_transforms(cfg):
    g = golden("stft")
    win, hop, nfft = cfg
    tag = f"{win}_{hop}_{nfft}"
    fwd, inv, window = O_stft.dft_bases(win, nfft)
    np.testing.assert_allclose(fwd[:, 0].norm(dim=1).numpy(), g[f"kw_norm_{tag}"], rtol=1e-6)
    np.testing.assert_array_equal(fwd[:3, 0].numpy(), g[f"kw_rows_{tag}"])
    np.testing.assert_allclose(inv[:, 0].norm(dim=1).numpy(), g[f"ki_norm_{tag}"], rtol=1e-5)
    np.testing.assert_allclose(inv[:3, 0].numpy(), g[f"ki_rows_{tag}"], rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(window[0, :, 0].numpy(), g[f"window_{tag}"])
    st, ist = O_stft.ConvSTFT(win, hop, nfft), O_stft.ConviSTFT(win, hop, nfft)
    x = torch.from_numpy(g[f"x_{tag}"])
    assert rel_l2(st(x).numpy(), g[f"spec_{tag}"]) < 1e-6
    s = torch.from_numpy(g[f"srand_{tag}"])
    assert rel_l2(ist(s).numpy(), g[f"irand_{tag}"]) < 1e-6
    assert rel_l2(ist(torch.from_numpy(g[f"spec_{tag}"])).numpy(), g[f"iself_{tag}"]) < 1e-6
    assert rel_l2(ist(s, output_length=2900).numpy(), g[f"ilen_{tag}"]) < 1e-6
    sr = s.clone().requires_grad_(True)
    (ist(sr) * torch.from_numpy(g[f"igout_{tag}"])).sum().backward()
    assert rel_l2(sr.grad.numpy(), g[f"igspec_{tag}"]) < 1e-6


def test_stft_mag_phase():
    g = golden("stft")
    st = O_stft.ConvSTFT(320, 160, 320, return_mag_phase=True)
    mag, ph = st(torch.from_numpy(g["mp_x"]))
    assert rel_l2(mag.numpy(), g["mp_mag"]) < 1e-6
    # phase is only defined where the magnitude is not ~0
    sel = g["mp_mag"] > 1e-3
    assert np.abs(ph.numpy()[sel] - g["mp_phase"][sel]).max() < 1e-4
    inv = O_stft.ConviSTFT(320, 160, 320)(mag, ph)
    assert rel_l2(inv.numpy(), g["mp_inv"]) < 1e-5


CONV_CASES = [
    ("enc", False, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
    ("padbias", False, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=True)),
    ("k7", False, 4, 2, 7, dict(padding=3, bias=False)),
    ("dec", True, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
    ("dccrn_dec", True, 8, 6, (5, 2), dict(stride=(2, 1), padding=(2, 0), output_padding=(1, 0), bias=True)),
    ("dcunet_dec", True, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=False)),
]


@pytest.mark.parametrize("i,case", list(enumerate(CONV_CASES)))
def test_complex_conv(i, case):
    g = golden("cconv")
    name, tr, cin, cout, k, kw = case
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, k, **kw), seed=i)
    x = torch.from_numpy(g[f"{name}_x"]).requires_grad_(True)
    y = m(x)
    assert rel_l2(y.detach().numpy(), g[f"{name}_y"]) < 1e-6
    (y * torch.from_numpy(g[f"{name}_gy"])).sum().backward()
    assert rel_l2(x.grad.numpy(), g[f"{name}_dx"]) < 1e-6
    assert rel_l2(m.real_conv.weight.grad.numpy(), g[f"{name}_dwr"]) < 1e-6
    assert rel_l2(m.imag_conv.weight.grad.numpy(), g[f"{name}_dwi"]) < 1e-6


@pytest.mark.parametrize("name,C,seed", [("c5", 10, 0), ("c1", 2, 1)])
def test_complex_batchnorm(name, C, seed):
    g = golden("cbn")
    m = paramfill.fill_(O_cnn.ComplexBatchNorm2d(C), seed=seed)
    np.testing.assert_array_equal(torch.cat([m.Wrr, m.Wri, m.Wii, m.Br, m.Bi]).detach().numpy(), g[f"{name}_params0"])
    x = torch.from_numpy(g[f"{name}_x"]).requires_grad_(True)
    y = m.train()(x)
    assert rel_l2(y.detach().numpy(), g[f"{name}_y"]) < 2e-6
    (y * torch.from_numpy(g[f"{name}_gy"])).sum().backward()
    assert rel_l2(x.grad.numpy(), g[f"{name}_dx"]) < 1e-5
    dp = torch.cat([m.Wrr.grad, m.Wri.grad, m.Wii.grad, m.Br.grad, m.Bi.grad]).numpy()
    assert rel_l2(dp, g[f"{name}_dparams"]) < 1e-5
    run = torch.cat([m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii]).detach().numpy()
    np.testing.assert_allclose(run, g[f"{name}_run1"], rtol=1e-5, atol=1e-6)
    assert int(m.num_batches_tracked) == 1
    m2 = paramfill.fill_(O_cnn.ComplexBatchNorm2d(C), seed=seed).eval()
    xe = torch.from_numpy(g[f"{name}_x"]).requires_grad_(True)
    ye = m2(xe)
    assert rel_l2(ye.detach().numpy(), g[f"{name}_yeval"]) < 1e-6
    (ye * torch.from_numpy(g[f"{name}_gy"])).sum().backward()
    assert rel_l2(xe.grad.numpy(), g[f"{name}_dxeval"]) < 1e-6


def test_ccbam_lstm_linear():
    g = golden("blocks")
    m = paramfill.fill_(O_ccbam.CCBAM(32, 16), seed=3)
    x = torch.from_numpy(g["ccbam_x"]).requires_grad_(True)
    y = m(x)
    assert rel_l2(y.detach().numpy(), g["ccbam_y"]) < 1e-6
    (y * torch.from_numpy(g["ccbam_gy"])).sum().backward()
    assert rel_l2(x.grad.numpy(), g["ccbam_dx"]) < 1e-5
    for n, p in m.named_parameters():
        assert rel_l2(p.grad.numpy(), g["ccbam_g_" + n]) < 1e-4, n
    lstm = paramfill.fill_(O_cnn.ComplexLSTM(16, 12, num_layers=2, batch_first=True), seed=4)
    assert rel_l2(lstm(torch.from_numpy(g["clstm_x"])).detach().numpy(), g["clstm_y"]) < 1e-6
    lin = paramfill.fill_(O_cnn.ComplexLinear(16, 8, bias=True), seed=5)
    assert rel_l2(lin(torch.from_numpy(g["clin_x"])).detach().numpy(), g["clin_y"]) < 1e-6


MODELS = [
    ("frcrn", lambda: O_models.FRCRN(320, 160, 640)),
    ("dccrn", lambda: O_models.DCCRN("dccrn-CL", 400, 100, 512)),
    ("dcunet16", lambda: O_models.DCUNet("dcunet16", 512, 128, 512)),
    ("carn", lambda: O_models.CARN(320, 160, 512)),
    ("gcarn", lambda: O_models.GCARN(320, 160, 512)),
    ("crn", lambda: O_models.CRN(320, 160, 320)),
]


@pytest.mark.parametrize("i,case", list(enumerate(MODELS)))
def test_model_forward(i, case):
    name, ctor = case
    g = golden(f"model_{name}")
    m = paramfill.fill_(ctor(), seed=20 + i)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        spec, wav = m.train()(x)
        assert rel_l2(spec.numpy(), g["spec_train"]) < 1e-5, "train spec"
        assert rel_l2(wav.numpy(), g["wav_train"]) < 1e-5, "train wav"
        spec, wav = m.eval()(x)
        assert rel_l2(spec.numpy(), g["spec_eval"]) < 1e-5, "eval spec"
        assert rel_l2(wav.numpy(), g["wav_eval"]) < 1e-5, "eval wav"


# drop-in constructor variants beyond the BASELINE configs (tests/golden/gen_golden.py
# variant_cases: same order, seeds 70 + i)
VARIANTS = [
    ("dccrn_r", lambda: O_models.DCCRN("dccrn-R", 400, 100, 512)),
    ("dccrn_c", lambda: O_models.DCCRN("dccrn-C", 400, 100, 512)),
    ("dccrn_bi", lambda: O_models.DCCRN("dccrn-CL", 400, 100, 512, bidirectional=True)),
    ("dccrn_real", lambda: O_models.DCCRN("dccrn-CL", 400, 100, 512, is_complex=False)),
    ("dcunet10", lambda: O_models.DCUNet("dcunet10", 512, 128, 512)),
    ("dcunet20", lambda: O_models.DCUNet("dcunet20", 512, 128, 512)),
    ("dcunet20_large", lambda: O_models.DCUNet("dcunet20-large", 1024, 256, 1024)),
]


@pytest.mark.parametrize("i,case", list(enumerate(VARIANTS)), ids=[v[0] for v in VARIANTS])
def test_variant_forward(i, case):
    name, ctor = case
    g = golden(f"variant_{name}")
    m = paramfill.fill_(ctor(), seed=70 + i)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        for mode in ("train", "eval"):
            spec, wav = (m.train() if mode == "train" else m.eval())(x)
            assert rel_l2(spec.numpy(), g[f"spec_{mode}"]) < 1e-5, (name, mode, "spec")
            assert rel_l2(wav.numpy(), g[f"wav_{mode}"]) < 1e-5, (name, mode, "wav")


def test_frcrn_train_step():
    g = golden("train_step_frcrn")
    m = paramfill.fill_(O_models.FRCRN(320, 160, 640), seed=30).train()
    names = [n for n, _ in m.named_parameters()]
    assert names == list(g["names"])
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    noisy, clean = torch.from_numpy(g["noisy"]), torch.from_numpy(g["clean"])
    _, wav = m(noisy[:, None, :])
    loss = O_train.si_snr_loss(O_train.pad_or_truncate_wav(wav, clean), clean)
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-4 * abs(float(g["loss"])) + 1e-5
    loss.backward()
    gn = torch.stack([p.grad.norm() for _, p in m.named_parameters()]).numpy()
    rel = np.abs(gn - g["grad_norms"]) / np.maximum(g["grad_norms"], 1e-12)
    assert np.median(rel) < 1e-4 and rel.max() < 5e-3, (np.median(rel), rel.max())
    total = torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
    assert abs(float(total) - float(g["grad_total_norm"])) < 1e-4 * float(g["grad_total_norm"])
    opt.step()
    heads = torch.stack([torch.nn.functional.pad(p.detach().flatten()[:16], (0, max(0, 16 - p.numel())))
                         for _, p in m.named_parameters()]).numpy()
    # Adam's first step moves each weight by ~lr*sign(g): where |g| is at the
    # rounding level the sign may differ, so allow a few 2*lr flips.
    d = np.abs(heads - g["param_heads"])
    assert d.max() <= 2.1e-3 and (d > 1e-5).mean() < 0.02, ((d > 1e-5).mean(), d.max())
