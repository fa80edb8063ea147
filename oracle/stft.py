"""Oracle ConvSTFT / ConviSTFT: the fixed-basis conv formulation.

Restates /root/reference/models/conv_stft.py (test infrastructure only).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from scipy.signal import get_window


def dft_bases(win: int, nfft: int, win_type: str = "hann"):
    """conv_stft.py:7-26. Windowed real-DFT analysis basis and its pinv
    synthesis basis, both built in float64 and rounded to float32.

    Analysis rows: cos(2*pi*k*n/N) for k = 0..N/2, then -sin(...) (numpy's
    rfft sign), each multiplied by the periodic window w[n], n < win.
    Synthesis rows: pinv(analysis_unwindowed)^T * w.
    """
    w = get_window(win_type, win, fftbins=True)                  # :10
    eye_rfft = np.fft.rfft(np.eye(nfft))[:win]                   # :11  [win, N/2+1]
    basis = np.concatenate([eye_rfft.real, eye_rfft.imag], axis=1).T   # :13-15 [N+2, win]
    synth = np.linalg.pinv(basis).T                              # :17-18
    fwd = torch.from_numpy((basis * w)[:, None, :].astype(np.float32))  # :20-24
    inv = torch.from_numpy((synth * w)[:, None, :].astype(np.float32))
    window = torch.from_numpy(w[None, :, None].astype(np.float32))      # :22,25
    return fwd, inv, window


class ConvSTFT(nn.Module):
    """conv_stft.py:29-66."""

    def __init__(self, window_size, hop_size, fft_size=None, win_type="hann",
                 center=True, return_mag_phase=False, fix=True):
        super().__init__()
        self.fft_size = window_size if fft_size is None else fft_size
        fwd, _, _ = dft_bases(window_size, self.fft_size, win_type)
        self.register_buffer("weight", fwd)                          # :40
        self.window_size, self.hop_size = window_size, hop_size
        self.center, self.return_mag_phase = center, return_mag_phase
        self.pad = self.fft_size // 2

    def forward(self, x):
        x = x.reshape((1, 1, -1) if x.dim() == 1 else (x.shape[0], 1, x.shape[-1]))   # :49-52
        if self.center:
            x = F.pad(x, (self.pad, self.pad), mode="reflect")      # :54-55
        spec = F.conv1d(x, self.weight.to(x.dtype), stride=self.hop_size)    # :56
        if not self.return_mag_phase:
            return spec
        half = self.fft_size // 2 + 1                                # :59-64
        re, im = spec[:, :half], spec[:, half:]
        return torch.sqrt(re * re + im * im), torch.atan2(im, re)


class ConviSTFT(nn.Module):
    """conv_stft.py:69-116."""

    def __init__(self, window_size, hop_size, fft_size=None, win_type="hann",
                 center=True, fix=True):
        super().__init__()
        self.fft_size = window_size if fft_size is None else fft_size
        _, inv, window = dft_bases(window_size, self.fft_size, win_type)
        self.register_buffer("weight", inv)                          # :80
        self.register_buffer("window", window)                       # :81
        self.register_buffer("enframe", torch.eye(window_size)[:, None, :])  # :82
        self.window_size, self.hop_size, self.center = window_size, hop_size, center
        self.pad = self.fft_size // 2

    def forward(self, inputs, phase=None, output_length=None):
        if phase is not None:                                        # :96-100
            inputs = torch.cat([inputs * torch.cos(phase), inputs * torch.sin(phase)], dim=1)
        wav = F.conv_transpose1d(inputs, self.weight.to(inputs.dtype), stride=self.hop_size)  # :101
        # OLA normaliser of window^2, recomputed per call in the reference (:104-105)
        w2 = (self.window.to(inputs.dtype) ** 2).expand(1, -1, inputs.shape[-1])
        coff = F.conv_transpose1d(w2, self.enframe.to(inputs.dtype), stride=self.hop_size)
        wav = wav / (coff + 1e-8)                                    # :106
        if self.center:                                              # :109-111
            wav = wav[..., self.pad:]
            if output_length is None:
                wav = wav[..., :-self.pad]
        if output_length is not None:                                # :113-114
            wav = wav[..., :output_length]
        return wav.squeeze(1)                                        # :116
