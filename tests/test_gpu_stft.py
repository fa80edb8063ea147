"""GPU parity: FFT-based ConvSTFT / ConviSTFT (csrc/stft.hip) vs reference
goldens (fp32, rel-L2 < 1e-5) for every window/hop/nfft config the models use."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2

pytestmark = pytest.mark.gpu

STFT_CONFIGS = [(320, 160, 640), (400, 100, 512), (512, 128, 512),
                (320, 160, 512), (320, 160, 320), (1024, 256, 1024)]


@pytest.mark.parametrize("cfg", STFT_CONFIGS)
def test_stft_istft_golden(cfg, gpu_device):
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    g = golden("stft")
    win, hop, nfft = cfg
    tag = f"{win}_{hop}_{nfft}"
    st = ConvSTFT(win, hop, nfft).cuda()
    ist = ConviSTFT(win, hop, nfft).cuda()
    np.testing.assert_array_equal(st.weight[:3, 0].cpu().numpy(), g[f"kw_rows_{tag}"])
    x = torch.from_numpy(g[f"x_{tag}"]).cuda()
    assert rel_l2(st(x).cpu().numpy(), g[f"spec_{tag}"]) < 1e-5
    s = torch.from_numpy(g[f"srand_{tag}"]).cuda()
    assert rel_l2(ist(s).cpu().numpy(), g[f"irand_{tag}"]) < 1e-5
    assert rel_l2(ist(torch.from_numpy(g[f"spec_{tag}"]).cuda()).cpu().numpy(), g[f"iself_{tag}"]) < 1e-5
    assert rel_l2(ist(s, output_length=2900).cpu().numpy(), g[f"ilen_{tag}"]) < 1e-5
    sr = s.clone().requires_grad_(True)
    (ist(sr) * torch.from_numpy(g[f"igout_{tag}"]).cuda()).sum().backward()
    assert rel_l2(sr.grad.cpu().numpy(), g[f"igspec_{tag}"]) < 1e-5


def test_stft_mag_phase_golden(gpu_device):
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    g = golden("stft")
    mag, ph = ConvSTFT(320, 160, 320, return_mag_phase=True).cuda()(torch.from_numpy(g["mp_x"]).cuda())
    assert rel_l2(mag.cpu().numpy(), g["mp_mag"]) < 1e-5
    sel = g["mp_mag"] > 1e-3
    d = np.angle(np.exp(1j * (ph.cpu().numpy()[sel].astype(np.float64) - g["mp_phase"][sel])))
    assert np.abs(d).max() < 1e-4   # compared on the circle (atan2 branch cut at +-pi)
    inv = ConviSTFT(320, 160, 320).cuda()(mag, ph)
    assert rel_l2(inv.cpu().numpy(), g["mp_inv"]) < 1e-5


def test_stft_roundtrip_full_size(gpu_device):
    """Size-independent property at the bench size (64 x 4 s): iSTFT(STFT(x)) = x."""
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    x = torch.randn(64, 64000, device="cuda") * 0.3
    st, ist = ConvSTFT(320, 160, 640).cuda(), ConviSTFT(320, 160, 640).cuda()
    spec = st(x)
    assert spec.shape == (64, 642, 403)
    y = ist(spec)
    assert y.shape == (64, 64000)
    assert rel_l2(y.cpu().numpy(), x.cpu().numpy()) < 2e-6


def test_stft_vs_oracle_4s(gpu_device):
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    from oracle import stft as O
    x = torch.randn(2, 64000) * 0.3
    ref = O.ConvSTFT(320, 160, 640)(x)
    out = ConvSTFT(320, 160, 640).cuda()(x.cuda()).cpu()
    assert rel_l2(out.numpy(), ref.numpy()) < 1e-5
    s = torch.randn(2, 642, 403)
    assert rel_l2(ConviSTFT(320, 160, 640).cuda()(s.cuda()).cpu().numpy(),
                  O.ConviSTFT(320, 160, 640)(s).numpy()) < 1e-5


@pytest.mark.parametrize("win,hop,nfft", [(256, 128, 256), (300, 150, 480), (400, 100, 400)])
def test_stft_istft_vs_oracle_more_plans(win, hop, nfft, gpu_device):
    """Compiled FFT plans (256, 400) and the runtime-plan path (480 = 4*4*2*3*5)
    against the oracle's DFT-basis conv1d restatement (conv_stft.py:48-116)."""
    from oracle import stft as O
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    torch.manual_seed(nfft)
    x = torch.randn(3, 8000) * 0.3
    ref = O.ConvSTFT(win, hop, nfft)(x)
    out = ConvSTFT(win, hop, nfft).cuda()(x.cuda()).cpu()
    assert rel_l2(out.numpy(), ref.numpy()) < 1e-5
    s = torch.randn_like(ref)
    assert rel_l2(ConviSTFT(win, hop, nfft).cuda()(s.cuda()).cpu().numpy(),
                  O.ConviSTFT(win, hop, nfft)(s).numpy()) < 1e-5


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-2), (torch.float16, 1.5e-3)])
@pytest.mark.parametrize("cfg", [(320, 160, 640), (400, 100, 512), (512, 128, 512)])
def test_stft_istft_low_precision_storage(cfg, dtype, tol, gpu_device):
    """bf16 / fp16 signals and spectra (model.to(bfloat16) / .half(), BASELINE configs 2, 3,
    5): the kernels read and write the storage type directly (fp32 arithmetic, fp32
    window / twiddle tables). Against the fp32 goldens on the rounded input, within the
    storage's rounding; the outputs are in the storage dtype."""
    from sehip.conv_stft import ConvSTFT, ConviSTFT
    g = golden("stft")
    win, hop, nfft = cfg
    tag = f"{win}_{hop}_{nfft}"
    st = ConvSTFT(win, hop, nfft).cuda().to(dtype)
    ist = ConviSTFT(win, hop, nfft).cuda().to(dtype)
    x = torch.from_numpy(g[f"x_{tag}"]).cuda().to(dtype)
    spec = st(x)
    assert spec.dtype == dtype
    ref = ConvSTFT(win, hop, nfft).cuda()(x.float())
    assert rel_l2(spec.float().cpu().numpy(), ref.cpu().numpy()) < tol
    assert rel_l2(spec.float().cpu().numpy(), g[f"spec_{tag}"]) < 2 * tol
    s = torch.from_numpy(g[f"srand_{tag}"]).cuda().to(dtype).requires_grad_(True)
    out = ist(s)
    assert out.dtype == dtype
    assert rel_l2(out.detach().float().cpu().numpy(), g[f"irand_{tag}"]) < 2 * tol
    (out * torch.from_numpy(g[f"igout_{tag}"]).cuda().to(dtype)).sum().backward()
    assert s.grad.dtype == dtype
    assert rel_l2(s.grad.float().cpu().numpy(), g[f"igspec_{tag}"]) < 2 * tol
