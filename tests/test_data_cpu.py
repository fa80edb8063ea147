"""CPU: the data path's host decisions draw the reference's random numbers
in the reference's order (mix_audio.py:87-121, audio_dataloader.py:32-48),
so a seeded run crops, pads, drops and picks SNRs as the reference would."""
import random

import torch

from oracle import data as OD


def test_spliter_plan_matches_oracle_draws():
    from sehip.data import AudioSpliter
    lengths = [40000, 15999, 16000, 31999, 32000, 64000, 7000, 52345] * 3
    plan = AudioSpliter(32000, 16000, rng=random.Random(9)).plan(lengths)
    rng = random.Random(9)
    for L, (keep, start) in zip(lengths, plan):
        s = {"mix": torch.arange(L, dtype=torch.float32)[None], "ref": []}
        out = OD.split(s, 32000, 16000, rng)
        assert keep == bool(out)
        if out:
            assert out[0]["mix"].shape[-1] == 32000
            if L >= 32000:
                assert out[0]["mix"][0, 0].item() == start


def test_oracle_mixer_realises_the_snr():
    g = torch.Generator().manual_seed(1)
    clean, noise = torch.randn(1, 16000, generator=g), torch.randn(1, 40000, generator=g)
    mixed, rep, snr, _ = OD.mix_one(clean, noise, random.Random(2))
    p = 10 * torch.log10(clean.pow(2).mean() / rep.pow(2).mean())
    assert abs(p.item() - snr) < 1e-3
    assert torch.allclose(mixed, clean + rep)
