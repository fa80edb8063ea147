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


def initialize_params(model, nonlinearity="relu"):
    """utils.py:47-84 (weight_norm=False, as train.py:38 calls it): kaiming-normal
    for every Conv1d/Conv2d/ConvTranspose1d/ConvTranspose2d/Linear weight (zero
    bias), xavier-uniform W_ih / orthogonal W_hh / zero biases for nn.LSTM, 1/0 for
    BatchNorm1d/2d. Returns the qualified names of the modules it touched, in
    visiting order (test infrastructure: the drop-in must expose the same ones)."""
    nn = torch.nn
    touched = []
    for name, module in model.named_modules():
        if isinstance(module, (nn.Conv1d, nn.Conv2d, nn.ConvTranspose1d, nn.ConvTranspose2d, nn.Linear)):
            nn.init.kaiming_normal_(module.weight.data, nonlinearity=nonlinearity)
            if module.bias is not None:
                nn.init.zeros_(module.bias.data)
        elif isinstance(module, nn.LSTM):
            for pname, param in module.named_parameters():
                if "weight_ih" in pname:
                    nn.init.xavier_uniform_(param.data)
                elif "weight_hh" in pname:
                    nn.init.orthogonal_(param.data)
                elif "bias" in pname:
                    nn.init.zeros_(param.data)
        elif isinstance(module, (nn.BatchNorm1d, nn.BatchNorm2d)):
            nn.init.constant_(module.weight.data, 1)
            nn.init.constant_(module.bias.data, 0)
        else:
            continue
        touched.append(name)
    return touched
