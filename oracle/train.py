"""Oracle training step: SI-SNR loss + backward + clip + AdamW.

Restates /root/reference/losses.py:62-84, utils.py:105-121 and the hot loop
of trainer.py:99-124 + 210-221 (test infrastructure only).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def si_snr_loss(est, tgt, zero_mean=False, eps=1e-8):
    """losses.py:62-84: -mean_b 10 log10(|s|^2+eps / |e-s|^2+eps)."""
    if zero_mean:
        est = est - est.mean(dim=1, keepdim=True)
        tgt = tgt - tgt.mean(dim=1, keepdim=True)
    dot = (est * tgt).sum(dim=1, keepdim=True)
    s = dot * tgt / torch.norm(tgt, dim=1, keepdim=True) ** 2
    num = torch.norm(s, dim=1) ** 2 + eps
    den = torch.norm(est - s, dim=1) ** 2 + eps
    return -torch.mean(10 * torch.log10(num / den))


def reshape_wav_to_mono(w):
    """utils.py:105-109."""
    return w.reshape(-1, w.shape[-1]) if w.dim() == 3 else w


def pad_or_truncate_wav(est, tgt):
    """utils.py:111-121."""
    le, lt = est.shape[-1], tgt.shape[-1]
    if le < lt:
        return F.pad(est, (0, lt - le))
    return est[:, :lt] if le > lt else est


def train_step(model, optimizer, noisy, clean, clip_norm=0.5):
    """trainer.py:99-124 + 210-221. Returns (loss, pre-clip total grad norm)."""
    _, wav = model(noisy)
    est = pad_or_truncate_wav(reshape_wav_to_mono(wav), reshape_wav_to_mono(clean))
    loss = si_snr_loss(est, reshape_wav_to_mono(clean))
    loss.backward()
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), clip_norm) if clip_norm else None
    optimizer.step()
    optimizer.zero_grad()
    return loss.detach(), total
