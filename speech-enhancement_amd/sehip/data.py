"""Synthetic noisy/clean utterance pairs generated on the device
(SURVEY.md §8d 'Synthetic inputs'; BASELINE.json metric: 4 s @ 16 kHz).

clean = peak-normalised sum of 3-5 harmonics (f0 ~ U[100, 300] Hz) under a
slow AM envelope + 0.05 N(0,1); noise = N(0,1); noisy = clean + g * noise at
an SNR drawn from U{-5..20} dB. Seeds: 2023 + rank * 1_000_003 + step
(2023 is the reference's unused hparams seed, hyperparams.py:12).
"""
from __future__ import annotations

import math

import torch


def synthetic_pairs(batch: int, length: int = 64000, sr: int = 16000, seed: int = 2023,
                    device="cuda", dtype=torch.float32):
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    f0 = torch.empty(batch, 1).uniform_(100.0, 300.0, generator=g)
    nh = torch.randint(3, 6, (batch, 1), generator=g)
    am_f = torch.empty(batch, 1).uniform_(1.0, 4.0, generator=g)
    phase = torch.empty(batch, 5).uniform_(0, 2 * math.pi, generator=g)
    snr_db = torch.randint(-5, 21, (batch, 1), generator=g).to(torch.float32)
    dev_g = torch.Generator(device=device).manual_seed(int(seed) + 7)
    t = torch.arange(length, device=device, dtype=dtype)[None] / sr
    f0, nh, am_f, phase, snr_db = (v.to(device) for v in (f0, nh, am_f, phase, snr_db))
    clean = torch.zeros(batch, length, device=device, dtype=dtype)
    for h in range(1, 6):
        on = (h <= nh).to(dtype)
        clean += on * torch.sin(2 * math.pi * h * f0 * t + phase[:, h - 1:h]) / h
    clean *= 0.6 + 0.4 * torch.sin(2 * math.pi * am_f * t)
    clean += 0.05 * torch.randn(batch, length, device=device, dtype=dtype, generator=dev_g)
    clean *= 0.5 / clean.abs().amax(dim=1, keepdim=True)
    noise = torch.randn(batch, length, device=device, dtype=dtype, generator=dev_g)
    p_c = clean.pow(2).mean(dim=1, keepdim=True)
    p_n = noise.pow(2).mean(dim=1, keepdim=True)
    gain = torch.sqrt(p_c / (p_n * 10 ** (snr_db / 10)))
    noisy = clean + gain * noise
    return noisy, clean
