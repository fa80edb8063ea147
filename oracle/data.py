"""Oracle for the data path (test infrastructure only): CPU restatements of
/root/reference/mix_audio.py:14-123 (get_rms, get_adjusted_rms, the mixing
loop of get_noisy_data) and audio_dataloader.py:29-50 (AudioSpliter.split)
plus default_collate, in torch fp32 on the CPU as the reference computes them.

Parity unpinned: mix_audio.py, audio_dataset.py and audio_dataloader.py import
torchaudio, which is absent here, so the reference cannot be run to make
fixtures; this restatement follows the source line by line and the GPU tests
(tests/test_gpu_data.py) compare the device kernels against it. The PCM16
float conversion follows torchaudio's documented normalisation (x / 32768 on
load); its save-side rounding (rint, clamp) is this build's choice.
"""
from __future__ import annotations

import random

import torch
import torch.nn.functional as F


def get_rms(signal):
    """mix_audio.py:14-15."""
    return torch.sqrt(torch.mean(signal ** 2, axis=-1, keepdim=True))


def get_adjusted_rms(clean_rms, snr):
    """mix_audio.py:17-18."""
    return clean_rms / 10 ** (snr / 20)


def mix_one(clean_amp, noise_amp, rng, noise_repeat=None):
    """One iteration of the loop at mix_audio.py:87-123 (clean_amp, noise_amp:
    [1, L] fp32 CPU tensors). Returns (mixed, repeat_noise, snr, noise_indices)."""
    if noise_amp.shape[1] > clean_amp.shape[1]:                       # :88-93
        start = rng.randint(0, noise_amp.shape[1] - clean_amp.shape[1])
        split_noise_amp = noise_amp[:, start:start + clean_amp.shape[1]]
    else:
        split_noise_amp = noise_amp[:]
    clean_rms = get_rms(clean_amp)                                     # :95-100
    noise_rms = get_rms(split_noise_amp)
    snr = rng.randint(-20, 20)
    adjusted_noise_rms = get_adjusted_rms(clean_rms, snr)
    adjusted_noise_amp = split_noise_amp * (adjusted_noise_rms / noise_rms)
    repeat_noise_amp = torch.zeros_like(clean_amp)                     # :102-121
    clean_length = clean_amp.shape[1]
    noise_length = adjusted_noise_amp.shape[1]
    max_repeat = clean_length // noise_length
    if noise_repeat is not None:
        noise_indices = []
        for _ in range(min(noise_repeat, max_repeat)):
            start = rng.randint(0, clean_length - noise_length)
            noise_indices.append([start, start + noise_length])
            repeat_noise_amp[:, start:start + noise_length] += adjusted_noise_amp
    else:
        end = max_repeat * noise_length
        noise_indices = [[i, i + noise_length] for i in range(0, end, noise_length)]
        repeat_noise_amp[:, 0:end] += adjusted_noise_amp.repeat((1, max_repeat))
    return clean_amp + repeat_noise_amp, repeat_noise_amp, snr, noise_indices   # :123


def split(sample, chunk_size, least_samples, rng):
    """AudioSpliter.split (audio_dataloader.py:29-50)."""
    sample_length = sample["mix"].shape[-1]
    if sample_length < least_samples:
        return []
    if sample_length < chunk_size:
        gap = chunk_size - sample_length
        return [{"mix": F.pad(sample["mix"], (0, gap)), "ref": [F.pad(r, (0, gap)) for r in sample["ref"]]}]
    start = rng.randint(0, sample_length - chunk_size)
    return [{"mix": sample["mix"][:, start:start + chunk_size],
             "ref": [r[:, start:start + chunk_size] for r in sample["ref"]]}]


def collate(samples, chunk_size, least_samples, rng):
    """AudioDataLoader._collate + default_collate (:68-78)."""
    items = []
    for s in samples:
        items += split(s, chunk_size, least_samples, rng)
    if not items:
        return []
    return {"mix": torch.stack([i["mix"] for i in items]),
            "ref": [torch.stack([i["ref"][j] for i in items]) for j in range(len(items[0]["ref"]))]}


def pcm16_to_float(x):
    return x.to(torch.float32) / 32768.0


def float_to_pcm16(x):
    return torch.clamp(torch.round(x * 32768.0), -32768, 32767).to(torch.int16)


def sinc_resample_kernel(orig_freq, new_freq, lowpass_filter_width=6, rolloff=0.99, dtype=torch.float32):
    """torchaudio.functional.resample's kernel (sinc_interp_hann, the default of
    torchaudio.transforms.Resample that mix_audio.py:71-77 uses), restated from
    torchaudio's published algorithm (torchaudio is absent here; parity unpinned):
    rates divided by their gcd; cut-off min(orig, new) * rolloff; per output phase a
    windowed sinc over 2 width + orig input taps. Returns (kernel [new, 1, K], width,
    orig', new')."""
    import math
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = torch.arange(-width, width + orig, dtype=dtype)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=dtype)[:, None, None] / new + idx
    t = (t * base).clamp(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    kern = torch.where(t == 0, torch.tensor(1.0, dtype=dtype), t.sin() / t)
    kern = kern * window * (base / orig)
    return kern, width, orig, new


def resample(waveform, orig_freq, new_freq):
    """torchaudio.functional.resample (sinc_interp_hann): pad width / width + orig,
    strided conv1d with the polyphase kernel, interleave phases, trim to
    ceil(new * L / orig)."""
    import math
    if orig_freq == new_freq:
        return waveform
    kern, width, orig, new = sinc_resample_kernel(orig_freq, new_freq, dtype=waveform.dtype)
    shape = waveform.shape
    w = waveform.reshape(-1, shape[-1])
    n, length = w.shape
    w = F.pad(w, (width, width + orig))
    out = F.conv1d(w[:, None], kern, stride=orig).transpose(1, 2).reshape(n, -1)
    out = out[..., :math.ceil(new * length / orig)]
    return out.reshape(shape[:-1] + out.shape[-1:])
