"""Data path on the device against the oracle
restatement of mix_audio.py:87-123 and audio_dataloader.py:29-50 (parity
unpinned: the reference modules import the absent torchaudio; see
oracle/data.py). Crop / pad and PCM16 conversion are data movement: bit-exact.
Mixing: the kernels sum squares in fp64 where torch sums fp32, so the scale
may differ in the last bits: rel 1e-6."""
import os
import random

import pytest
import torch

from oracle import data as OD

pytestmark = pytest.mark.gpu


def _signals(Lc, Ln, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(Lc) / 16000.0
    clean = (0.3 * torch.sin(2 * torch.pi * 220 * t) + 0.05 * torch.randn(Lc, generator=g))[None]
    noise = torch.randn(1, Ln, generator=g) * 0.7
    return clean, noise


@pytest.mark.parametrize("Lc,Ln,noise_repeat", [(16000, 48000, None), (16000, 5000, None), (16000, 5000, 2),
                                                (12000, 12000, None), (16000, 3999, 3), (8000, 20000, 1)])
def test_get_noisy_data_vs_oracle(Lc, Ln, noise_repeat, gpu_device):
    from sehip import data as D
    clean, noise = _signals(Lc, Ln, seed=Lc + Ln)
    k = 6
    c, n, out = D.get_noisy_data(clean.to(gpu_device), noise.to(gpu_device), noise_repeat=noise_repeat, k=k,
                                 rng=random.Random(11))
    rng = random.Random(11)
    for i in range(k):
        mixed, rep, snr, idx = OD.mix_one(clean, noise, rng, noise_repeat)
        assert out["snr"][i] == snr and out["noise_indices"][i] == idx
        got_rep, got_mix = out["repeat_noise"][i].cpu(), out["mixed_output"][i].cpu()
        assert torch.equal(got_rep == 0, rep == 0)                     # the same samples carry noise
        assert ((got_rep - rep).norm() / rep.norm()).item() < 1e-6
        assert ((got_mix - mixed).norm() / mixed.norm()).item() < 1e-6
        # realised SNR of the mix equals the drawn one (10 log10 of clean / noise power)
        if noise_repeat is None and Ln >= Lc:
            p = 10 * torch.log10(clean.pow(2).mean() / got_rep.pow(2).mean())
            assert abs(p.item() - snr) < 1e-3


@pytest.mark.parametrize("chunk,least", [(32000, 16000), (8000, 4000)])
def test_collate_crop_pad_bit_exact(chunk, least, gpu_device):
    """Ragged utterances (dropped, padded, exact-length and cropped) through the
    device collation: identical to the oracle's split + default_collate."""
    from sehip import data as D
    g = torch.Generator().manual_seed(3)
    lengths = [40000, 15999, 16000, 31999, 32000, 64000, 7000, 52345]
    samples = [{"mix": torch.randn(1, L, generator=g), "ref": [torch.randn(1, L, generator=g) for _ in range(2)]}
               for L in lengths]
    ref = OD.collate(samples, chunk, least, random.Random(5))
    dev = [{"mix": s["mix"].to(gpu_device), "ref": [r.to(gpu_device) for r in s["ref"]]} for s in samples]
    got = D.AudioSpliter(chunk, least, rng=random.Random(5)).collate(dev)
    assert got["mix"].shape == ref["mix"].shape
    assert torch.equal(got["mix"].cpu(), ref["mix"])
    for a, b in zip(got["ref"], ref["ref"]):
        assert torch.equal(a.cpu(), b)


def test_collate_all_dropped_is_empty(gpu_device):
    from sehip import data as D
    s = [{"mix": torch.randn(1, 100, device=gpu_device), "ref": [torch.randn(1, 100, device=gpu_device)]}]
    assert D.AudioSpliter(32000, 16000).collate(s) == []


def test_pcm16_round_trip_bit_exact(tmp_path, gpu_device):
    from sehip import data as D
    g = torch.Generator().manual_seed(4)
    pcm = torch.randint(-32768, 32768, (2, 12345), generator=g, dtype=torch.int32).to(torch.int16)
    x = D.pcm16_to_float(pcm.to(gpu_device))
    assert torch.equal(x.cpu(), OD.pcm16_to_float(pcm))
    assert torch.equal(D.float_to_pcm16(x).cpu(), pcm)                 # exact inverse on the grid
    y = torch.randn(3, 1000, generator=g) * 0.7
    y[0, :4] = torch.tensor([1.5, -1.5, 1.0, -1.0])                     # clamping at both ends
    assert torch.equal(D.float_to_pcm16(y.to(gpu_device)).cpu(), OD.float_to_pcm16(y))
    D.save_wav(tmp_path / "a.wav", x, 16000)
    back, sr = D.load_wav(tmp_path / "a.wav", gpu_device)
    assert sr == 16000 and torch.equal(back.cpu(), x.cpu())


@pytest.mark.parametrize("orig,new", [(48000, 16000), (44100, 16000), (8000, 16000), (22050, 16000),
                                      (16000, 16000)])
def test_resample_vs_oracle(orig, new, gpu_device):
    """se_resample (mix_audio.py:71-77's torchaudio Resample, sinc_interp_hann) against
    the oracle's restatement of torchaudio.functional.resample (conv1d form): same
    length, rel-L2 < 1e-6 (the taps are summed in another order)."""
    from sehip import data as D
    g = torch.Generator().manual_seed(orig)
    x = torch.randn(3, orig // 2 + 17, generator=g)
    got = D.resample(x.to(gpu_device), orig, new).cpu()
    ref = OD.resample(x, orig, new)
    assert got.shape == ref.shape
    assert ((got - ref).norm() / ref.norm()).item() < 1e-6


def test_resample_keeps_a_passband_tone(gpu_device):
    """A 440 Hz tone at 48 kHz resampled to 16 kHz is the 440 Hz tone at 16 kHz
    (away from the edges, where the filter sees the zero padding)."""
    from sehip import data as D
    t48 = torch.arange(48000, dtype=torch.float64) / 48000
    t16 = torch.arange(16000, dtype=torch.float64) / 16000
    y = D.resample(torch.sin(2 * torch.pi * 440 * t48).float().to(gpu_device), 48000, 16000).cpu().double()
    ref = torch.sin(2 * torch.pi * 440 * t16)
    assert (y[200:-200] - ref[200:-200]).abs().max().item() < 2e-3


def test_get_noisy_data_from_wav_paths(tmp_path, gpu_device):
    """The reference's call form (mix_audio.py:20-31): wav paths at other rates and
    stereo, save=True. Stereo is averaged to mono, both resampled to 16 kHz, k mixes
    returned under the reference's keys and written as PCM16 wavs named
    <clean>_<noise>_{mix,clean,noise}_<i>.wav."""
    from sehip import data as D
    g = torch.Generator().manual_seed(21)
    clean = (torch.randn(2, 24000, generator=g) * 0.1).clamp(-1, 1)   # stereo, 1 s at 24 kHz
    noise = (torch.randn(1, 8820, generator=g) * 0.1).clamp(-1, 1)    # mono, 0.4 s at 22.05 kHz
    D.save_wav(tmp_path / "c.wav", clean.to(gpu_device), 24000)
    D.save_wav(tmp_path / "n.wav", noise.to(gpu_device), 22050)
    out_dirs = [str(tmp_path / d) for d in ("mix", "clean", "noise")]
    c, n, outputs = D.get_noisy_data(str(tmp_path / "c.wav"), str(tmp_path / "n.wav"), *out_dirs, k=3, save=True,
                                     rng=random.Random(4))
    cl, _ = D.load_wav(tmp_path / "c.wav", gpu_device)
    ref_c = OD.resample(cl.cpu().mean(dim=0, keepdim=True), 24000, 16000)
    assert c.shape == (1, 16000) and n.shape == (1, 6400)
    assert ((c.cpu() - ref_c).norm() / ref_c.norm()).item() < 1e-6
    assert sorted(outputs) == ["adjusted_noise", "mixed_output", "noise_indices", "repeat_noise", "snr"]
    assert all(len(v) == 3 for v in outputs.values())
    assert outputs["mixed_output"][0].shape == (1, 16000)
    for d, kind in zip(out_dirs, ("mix", "clean", "noise")):
        for i in range(3):
            w, sr = D.load_wav(os.path.join(d, f"c_n_{kind}_{i}.wav"), gpu_device)
            assert sr == 16000 and w.shape == (1, 16000)


def test_audio_data_loader_matches_oracle_collate(gpu_device):
    """AudioDataLoader(dataset, chunk_size, least_samples, batch_size=...)
    (audio_dataloader.py:52-81): a DataLoader over ragged items, each batch cropped /
    padded on the device; batch for batch equal to the oracle's split +
    default_collate with the same random draws."""
    from sehip import data as D
    g = torch.Generator().manual_seed(6)
    lengths = [40000, 15999, 16000, 31999, 32000, 64000, 7000, 52345, 33000, 12000]
    items = [{"mix": torch.randn(1, L, generator=g), "ref": [torch.randn(1, L, generator=g)]} for L in lengths]
    loader = D.AudioDataLoader(items, chunk_size=32000, least_samples=16000, rng=random.Random(8), batch_size=4,
                               num_workers=0)
    assert len(loader) == len(items)
    rng = random.Random(8)
    got = list(loader)
    ref = [OD.collate(items[i:i + 4], 32000, 16000, rng) for i in range(0, len(items), 4)]
    ref = [r for r in ref if r]
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert torch.equal(a["mix"].cpu(), b["mix"]) and torch.equal(a["ref"][0].cpu(), b["ref"][0])
