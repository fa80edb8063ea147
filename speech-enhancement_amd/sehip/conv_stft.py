"""ConvSTFT / ConviSTFT on the HIP path.

Drop-in for /root/reference/models/conv_stft.py: same constructor/forward
signatures and the same state_dict buffers (``weight`` for the analysis
module; ``weight``, ``window``, ``enframe`` for the synthesis module), so a
reference checkpoint loads unchanged. The buffers are kept for compatibility
only — the kernels (csrc/stft.hip) evaluate the same linear maps with packed
real FFTs and never read the [N+2, 1, win] bases.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from scipy.signal import get_window

from . import functional as F


def _analysis_window(win_type: str, win: int) -> np.ndarray:
    return get_window(win_type, win, fftbins=True)          # conv_stft.py:10


def _basis(win: int, nfft: int, win_type: str, inverse: bool):
    """The reference's [N+2, 1, win] fp32 basis (conv_stft.py:7-26), built in
    float64 only to fill the state_dict buffer."""
    w = _analysis_window(win_type, win)
    cols = np.fft.rfft(np.eye(nfft))[:win]
    k = np.concatenate([cols.real, cols.imag], axis=1).T
    if inverse:
        k = np.linalg.pinv(k).T
    return torch.from_numpy((k * w)[:, None, :].astype(np.float32)), w


def _twiddles(nfft: int) -> torch.Tensor:
    ang = 2.0 * np.pi * np.arange(nfft) / nfft
    return torch.from_numpy(np.stack([np.cos(ang), -np.sin(ang)], axis=1).astype(np.float32).reshape(-1))


class _KernelTables(nn.Module):
    """Keeps the kernels' private fp32 tables (window, twiddles) in fp32 when the
    module is cast (model.half() / .to(bfloat16), as the reference's low-precision
    configs do): the state_dict buffers follow the cast like the reference's, the
    tables the kernels read do not. bf16 / fp16 signals and spectra are read and
    written in their own dtype by the kernels (SE_DTYPE_*), fp32 arithmetic."""

    _tables = ("_win", "_tw")

    def _apply(self, fn, *args, **kwargs):
        keep = {n: getattr(self, n).detach().cpu().float() for n in self._tables}
        super()._apply(fn, *args, **kwargs)
        for n, v in keep.items():
            buf = getattr(self, n)
            setattr(self, n, v.to(buf.device))
        return self


class ConvSTFT(_KernelTables):
    """conv_stft.py:29-66 (analysis)."""

    def __init__(self, window_size, hop_size, fft_size=None, win_type="hann", center=True,
                 return_mag_phase=False, fix=True):
        super().__init__()
        self.fft_size = window_size if fft_size is None else fft_size
        weight, w = _basis(window_size, self.fft_size, win_type, inverse=False)
        self.register_buffer("weight", weight)
        self.register_buffer("_win", torch.from_numpy(w.astype(np.float32)), persistent=False)
        self.register_buffer("_tw", _twiddles(self.fft_size), persistent=False)
        self.hop_size, self.window_size = hop_size, window_size
        self.center, self.return_mag_phase = center, return_mag_phase
        self.pad = self.fft_size // 2

    def forward(self, inputs):
        if inputs.dim() == 1:
            x = inputs[None]
        elif inputs.dim() == 2:
            x = inputs
        elif inputs.dim() == 3 and inputs.shape[1] == 1:
            x = inputs[:, 0]
        else:
            raise RuntimeError(f"ConvSTFT expects [L], [B, L] or [B, 1, L], got {tuple(inputs.shape)}")
        if self.center and x.shape[-1] <= self.pad:
            raise RuntimeError(f"reflect padding {self.pad} needs an input longer than {self.pad}")
        return F.stft(x, self._win, self._tw, self.window_size, self.hop_size, self.fft_size,
                      self.center, self.return_mag_phase)


class ConviSTFT(_KernelTables):
    """conv_stft.py:69-116 (synthesis with the pinv basis + window^2 OLA)."""

    def __init__(self, window_size, hop_size, fft_size=None, win_type="hann", center=True, fix=True):
        super().__init__()
        self.fft_size = window_size if fft_size is None else fft_size
        weight, w = _basis(window_size, self.fft_size, win_type, inverse=True)
        self.register_buffer("weight", weight)
        self.register_buffer("window", torch.from_numpy(w.astype(np.float32))[None, :, None])
        self.register_buffer("enframe", torch.eye(window_size)[:, None, :])
        self.register_buffer("_win", torch.from_numpy(w.astype(np.float32)), persistent=False)
        self.register_buffer("_tw", _twiddles(self.fft_size), persistent=False)
        self.hop_size, self.window_size, self.center = hop_size, window_size, center
        self.pad = self.fft_size // 2

    def forward(self, inputs, phase=None, output_length=None):
        if phase is not None:                                   # conv_stft.py:96-100
            inputs = torch.cat([inputs * torch.cos(phase), inputs * torch.sin(phase)], dim=1)
        t = inputs.shape[-1]
        full = (t - 1) * self.hop_size + self.window_size       # conv_transpose1d length
        if self.center:                                         # conv_stft.py:109-114
            offset = self.pad
            n = full - 2 * self.pad if output_length is None else min(output_length, full - self.pad)
        else:
            offset = 0
            n = full if output_length is None else min(output_length, full)
        return F.istft(inputs, self._win, self._tw, self.window_size, self.hop_size,
                       self.fft_size, offset, max(n, 0))
