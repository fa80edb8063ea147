"""Training losses (drop-in for /root/reference/losses.py). Plain PyTorch on
the device: a [B, L] reduction is negligible next to the conv stack."""
from __future__ import annotations

import torch


def SI_SNR_loss(estimate, target, zero_mean=False, eps=1e-8):
    """losses.py:62-84: negative mean scale-invariant SNR in dB."""
    if zero_mean:
        estimate = estimate - estimate.mean(dim=1, keepdim=True)
        target = target - target.mean(dim=1, keepdim=True)
    t_energy = target.pow(2).sum(dim=1, keepdim=True)
    proj = (estimate * target).sum(dim=1, keepdim=True) * target / t_energy
    signal = proj.pow(2).sum(dim=1) + eps
    noise = (estimate - proj).pow(2).sum(dim=1) + eps
    return -torch.mean(10 * torch.log10(signal / noise))


def SDR_loss(estimate, target, eps=1e-8):
    """losses.py:4-17: -mean 10 log10((|t|^2+eps) / (|t-e|^2+eps))."""
    t = target.pow(2).sum(dim=1) + eps
    e = (target - estimate).pow(2).sum(dim=1) + eps
    return -torch.mean(10 * torch.log10(t / e))


def reshape_wav_to_mono(wav):
    """utils.py:105-109."""
    if wav.dim() == 3:
        b, c, n = wav.shape
        wav = wav.reshape(b * c, n)
    return wav


def pad_or_truncate_wav(estimate_wav, target_wav):
    """utils.py:111-121."""
    le, lt = estimate_wav.shape[-1], target_wav.shape[-1]
    if le < lt:
        return torch.nn.functional.pad(estimate_wav, (0, lt - le))
    if le > lt:
        return estimate_wav[:, :lt]
    return estimate_wav
