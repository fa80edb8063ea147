"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

It imports shs2783/Speech-Enhancement from /root/reference exactly the way
train.py does (``models`` on sys.path, ops imported as top-level modules,
SURVEY.md §1 import quirk), fills every model with the name-keyed recipe of
paramfill.py and stores inputs + outputs as small compressed .npz files.
Nothing from the reference's source is copied into the fixtures: they hold
numbers only.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REF, "models"))

import paramfill  # noqa: E402

import conv_stft as R_stft  # noqa: E402
from modules import complex_nn as R_cnn  # noqa: E402
from modules import ccbam as R_ccbam  # noqa: E402
import losses as R_losses  # noqa: E402
import _2206_07293_frcrn as R_frcrn  # noqa: E402
import _2008_00264_dccrn as R_dccrn  # noqa: E402
import _1903_03107_dcunet as R_dcunet  # noqa: E402
import _2104_05267_carn as R_carn  # noqa: E402
import _1809_01405_crn as R_crn  # noqa: E402

torch.set_num_threads(8)
OUT = HERE


def save(name, **arrays):
    arrays = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
              for k, v in arrays.items()}
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
    size = os.path.getsize(os.path.join(OUT, name + ".npz"))
    print(f"{name}.npz  {size/1024:.0f} KiB  keys={sorted(arrays)}")


def randn(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


STFT_CONFIGS = [(320, 160, 640), (400, 100, 512), (512, 128, 512),
                (320, 160, 512), (320, 160, 320), (1024, 256, 1024)]


def gen_stft():
    out = {}
    for i, (win, hop, nfft) in enumerate(STFT_CONFIGS):
        tag = f"{win}_{hop}_{nfft}"
        x = randn(2 if i == 0 else 1, 3000, seed=100 + i, scale=0.3)
        stft = R_stft.ConvSTFT(win, hop, nfft)
        istft = R_stft.ConviSTFT(win, hop, nfft)
        spec = stft(x)
        out[f"x_{tag}"] = x
        out[f"spec_{tag}"] = spec
        # basis pinning: row norms of both bases + their first 3 rows
        out[f"kw_norm_{tag}"] = stft.weight[:, 0, :].norm(dim=1)
        out[f"kw_rows_{tag}"] = stft.weight[:3, 0, :]
        out[f"ki_norm_{tag}"] = istft.weight[:, 0, :].norm(dim=1)
        out[f"ki_rows_{tag}"] = istft.weight[:3, 0, :]
        out[f"window_{tag}"] = istft.window[0, :, 0]
        # inverse of a random (non-consistent) spectrum, and of the true one
        T = spec.shape[-1]
        s_rand = randn(x.shape[0], nfft + 2, T, seed=200 + i)
        out[f"srand_{tag}"] = s_rand
        out[f"irand_{tag}"] = istft(s_rand)
        out[f"iself_{tag}"] = istft(spec)
        out[f"ilen_{tag}"] = istft(s_rand, output_length=2900)
        # adjoint (gradient of a random projection of the inverse)
        s_req = s_rand.clone().requires_grad_(True)
        w = istft(s_req)
        gw = randn(*w.shape, seed=300 + i)
        (w * gw).sum().backward()
        out[f"igout_{tag}"] = gw
        out[f"igspec_{tag}"] = s_req.grad
    # magnitude / phase API (CRN, conv_stft.py:58-64, 96-100)
    x = randn(2, 4000, seed=150, scale=0.3)
    stft = R_stft.ConvSTFT(320, 160, 320, return_mag_phase=True)
    istft = R_stft.ConviSTFT(320, 160, 320)
    mag, ph = stft(x)
    out["mp_x"], out["mp_mag"], out["mp_phase"] = x, mag, ph
    out["mp_inv"] = istft(mag, ph)
    save("stft", **out)


CONV_CASES = [
    # name, transposed, cin, cout, kernel, kwargs, input shape
    ("enc", False, 16, 12, (5, 2), dict(stride=(2, 1), bias=False), (2, 16, 21, 13)),
    ("padbias", False, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=True), (2, 8, 17, 11)),
    ("k7", False, 4, 2, 7, dict(padding=3, bias=False), (2, 4, 9, 10)),
    ("dec", True, 16, 12, (5, 2), dict(stride=(2, 1), bias=False), (2, 16, 7, 9)),
    ("dccrn_dec", True, 8, 6, (5, 2), dict(stride=(2, 1), padding=(2, 0), output_padding=(1, 0), bias=True), (2, 8, 6, 7)),
    ("dcunet_dec", True, 8, 6, (5, 3), dict(stride=(2, 2), padding=(2, 1), bias=False), (2, 8, 6, 5)),
]


def gen_cconv():
    out = {}
    for i, (name, tr, cin, cout, k, kw, shape) in enumerate(CONV_CASES):
        cls = R_cnn.ComplexConvTranspose2d if tr else R_cnn.ComplexConv2d
        m = paramfill.fill_(cls(cin, cout, k, **kw), seed=i)
        x = randn(*shape, seed=400 + i).requires_grad_(True)
        y = m(x)
        gy = randn(*y.shape, seed=500 + i)
        (y * gy).sum().backward()
        out[f"{name}_x"], out[f"{name}_y"], out[f"{name}_gy"] = x, y, gy
        out[f"{name}_dx"] = x.grad
        out[f"{name}_dwr"] = m.real_conv.weight.grad
        out[f"{name}_dwi"] = m.imag_conv.weight.grad
        if m.real_conv.bias is not None:
            out[f"{name}_dbr"] = m.real_conv.bias.grad
            out[f"{name}_dbi"] = m.imag_conv.bias.grad
    # real conv (FRCRN final_conv, frcrn.py:115)
    m = paramfill.fill_(torch.nn.Conv2d(16, 2, (1, 2), bias=False), seed=9)
    x = randn(2, 16, 7, 9, seed=490).requires_grad_(True)
    y = m(x)
    gy = randn(*y.shape, seed=590)
    (y * gy).sum().backward()
    out.update(real_x=x, real_y=y, real_gy=gy, real_dx=x.grad, real_dw=m.weight.grad)
    save("cconv", **out)


def gen_cbn():
    out = {}
    for name, C, shape, seed in [("c5", 10, (4, 10, 7, 9), 0), ("c1", 2, (3, 2, 5, 11), 1)]:
        x = randn(*shape, seed=600 + seed, scale=1.5)
        x = x + torch.linspace(-0.5, 0.5, C).view(1, C, 1, 1)
        # train mode: batch statistics + running update
        m = paramfill.fill_(R_cnn.ComplexBatchNorm2d(C), seed=seed)
        out[f"{name}_params0"] = torch.cat([m.Wrr, m.Wri, m.Wii, m.Br, m.Bi]).detach()
        out[f"{name}_run0"] = torch.cat([m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii]).detach()
        xt = x.clone().requires_grad_(True)
        y = m.train()(xt)
        gy = randn(*y.shape, seed=700 + seed)
        (y * gy).sum().backward()
        out[f"{name}_x"], out[f"{name}_y"], out[f"{name}_gy"], out[f"{name}_dx"] = x, y, gy, xt.grad
        out[f"{name}_dparams"] = torch.cat([m.Wrr.grad, m.Wri.grad, m.Wii.grad, m.Br.grad, m.Bi.grad])
        out[f"{name}_run1"] = torch.cat([m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii]).detach()
        # eval mode with the filled (not updated) running stats
        m2 = paramfill.fill_(R_cnn.ComplexBatchNorm2d(C), seed=seed)
        xe = x.clone().requires_grad_(True)
        ye = m2.eval()(xe)
        (ye * gy).sum().backward()
        out[f"{name}_yeval"], out[f"{name}_dxeval"] = ye, xe.grad
        out[f"{name}_dparamseval"] = torch.cat([m2.Wrr.grad, m2.Wri.grad, m2.Wii.grad, m2.Br.grad, m2.Bi.grad])
    save("cbn", **out)


def gen_blocks():
    out = {}
    # CCBAM (ccbam.py:88-106) fwd + bwd
    m = paramfill.fill_(R_ccbam.CCBAM(32, 16), seed=3)
    x = randn(2, 32, 9, 11, seed=800).requires_grad_(True)
    y = m(x)
    gy = randn(*y.shape, seed=801)
    (y * gy).sum().backward()
    out.update(ccbam_x=x, ccbam_y=y, ccbam_gy=gy, ccbam_dx=x.grad)
    for n, p in m.named_parameters():
        out["ccbam_g_" + n] = p.grad
    # ComplexLSTM (complex_nn.py:115-145)
    lstm = paramfill.fill_(R_cnn.ComplexLSTM(16, 12, num_layers=2, batch_first=True), seed=4)
    xl = randn(2, 7, 16, seed=802)
    out.update(clstm_x=xl, clstm_y=lstm(xl))
    # ComplexLinear (complex_nn.py:93-113)
    lin = paramfill.fill_(R_cnn.ComplexLinear(16, 8, bias=True), seed=5)
    out.update(clin_x=xl, clin_y=lin(xl))
    save("blocks", **out)


def model_cases():
    return [
        ("frcrn", lambda: R_frcrn.FRCRN(320, 160, 640)),
        ("dccrn", lambda: R_dccrn.DCCRN("dccrn-CL", 400, 100, 512)),
        ("dcunet16", lambda: R_dcunet.DCUNet("dcunet16", 512, 128, 512)),  # needs L=32000 (see below)
        ("carn", lambda: R_carn.CARN(320, 160, 512)),
        ("gcarn", lambda: R_carn.GCARN(320, 160, 512)),
        ("crn", lambda: R_crn.CRN(320, 160, 320)),
    ]


def gen_models():
    noisy, _ = paramfill.structured_pair(2, 16000, seed=11)
    noisy2, _ = paramfill.structured_pair(1, 32000, seed=13)
    for i, (name, ctor) in enumerate(model_cases()):
        # DCUNet's crop (dcunet.py:141-146) only trims, so its frame count must
        # survive the stride pattern: 2 s (T=251) does, 1 s (T=126) does not.
        x = torch.from_numpy(noisy2 if name == "dcunet16" else noisy)
        out = {"x": x}
        m = paramfill.fill_(ctor(), seed=20 + i)
        with torch.no_grad():
            spec, wav = m.train()(x)
            out["spec_train"], out["wav_train"] = spec, wav
            spec, wav = m.eval()(x)
            out["spec_eval"], out["wav_eval"] = spec, wav
        save(f"model_{name}", **out)


def variant_cases():
    """Drop-in constructor variants beyond the BASELINE configs:
    (name, reference constructor, input length, batch). DCCRN masks 'R' / 'C'
    (_2008_00264_dccrn.py:127-132,188-193) and bidirectional=True (:124,143, LSTMBlock
    :60-64); DCUNet-10 / -20 / -20-large (architectures.py:55-98), the last at the
    reference's own test.py settings (1024/256/1024, 2 s, test.py:8-19); the real-valued
    (is_complex=False) DCCRN."""
    return [
        ("dccrn_r", lambda: R_dccrn.DCCRN("dccrn-R", 400, 100, 512), 16000, 1),
        ("dccrn_c", lambda: R_dccrn.DCCRN("dccrn-C", 400, 100, 512), 16000, 1),
        ("dccrn_bi", lambda: R_dccrn.DCCRN("dccrn-CL", 400, 100, 512, bidirectional=True), 16000, 1),
        ("dccrn_real", lambda: R_dccrn.DCCRN("dccrn-CL", 400, 100, 512, is_complex=False), 16000, 1),
        ("dcunet10", lambda: R_dcunet.DCUNet("dcunet10", 512, 128, 512), 32000, 1),
        ("dcunet20", lambda: R_dcunet.DCUNet("dcunet20", 512, 128, 512), 32000, 1),
        ("dcunet20_large", lambda: R_dcunet.DCUNet("dcunet20-large", 1024, 256, 1024), 32000, 1),
    ]


def gen_variants(only=None):
    for i, (name, ctor, L, B) in enumerate(variant_cases()):
        if only and name not in only:
            continue
        noisy, _ = paramfill.structured_pair(B, L, seed=60 + i)
        x = torch.from_numpy(noisy)
        out = {"x": x}
        m = paramfill.fill_(ctor(), seed=70 + i)
        with torch.no_grad():
            spec, wav = m.train()(x)
            out["spec_train"], out["wav_train"] = spec, wav
            spec, wav = m.eval()(x)
            out["spec_eval"], out["wav_eval"] = spec, wav
        save(f"variant_{name}", **out)


def gen_train_step():
    """One FRCRN training step exactly as trainer.py:99-124 + 210-221."""
    noisy, clean = paramfill.structured_pair(2, 16000, seed=12)
    noisy, clean = torch.from_numpy(noisy), torch.from_numpy(clean)
    m = paramfill.fill_(R_frcrn.FRCRN(320, 160, 640), seed=30).train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    spec, wav = m(noisy[:, None, :])
    est = wav  # reshape_wav_to_mono is a no-op on [B, L] (utils.py:105-109)
    tgt = clean
    if est.shape[-1] < tgt.shape[-1]:
        est = torch.nn.functional.pad(est, (0, tgt.shape[-1] - est.shape[-1]))
    loss = R_losses.SI_SNR_loss(est, tgt)
    loss.backward()
    names = [n for n, _ in m.named_parameters()]
    grads = [p.grad.detach().clone() for _, p in m.named_parameters()]
    total = torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
    opt.step()
    out = {"noisy": noisy, "clean": clean, "loss": loss.detach(), "wav": wav.detach(),
           "grad_total_norm": total, "names": np.array(names)}
    out["grad_norms"] = torch.stack([g.norm() for g in grads])
    out["grad_heads"] = torch.stack([torch.nn.functional.pad(g.flatten()[:16], (0, max(0, 16 - g.numel())))
                                     for g in grads])
    out["param_sums"] = torch.stack([p.detach().double().sum() for _, p in m.named_parameters()])
    out["param_heads"] = torch.stack([torch.nn.functional.pad(p.detach().flatten()[:16], (0, max(0, 16 - p.numel())))
                                      for _, p in m.named_parameters()])
    run = []
    for n, b in m.named_buffers():
        if n.split(".")[-1] in ("RMr", "RMi", "RVrr", "RVri", "RVii"):
            run.append(b.detach().flatten())
    out["running"] = torch.cat(run)
    save("train_step_frcrn", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["stft", "cconv", "cbn", "blocks", "models", "train", "variants"]
    torch.manual_seed(0)
    if "stft" in which: gen_stft()
    if "cconv" in which: gen_cconv()
    if "cbn" in which: gen_cbn()
    if "blocks" in which: gen_blocks()
    if "models" in which: gen_models()
    if "train" in which: gen_train_step()
    if "variants" in which: gen_variants()
