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


# --------------------------------------------------------------------------
# Real-data path: the reference's mixer and collation
# with the per-sample work on the device (csrc/data.hip). The random draws are
# made on the host with a `random.Random` in the reference's order, so a seeded
# run draws what the reference would; the kernels then mix / crop / pad.
# --------------------------------------------------------------------------
import os
import random as _random
import wave as _wave

from . import _native as N


def get_rms(signal: torch.Tensor) -> torch.Tensor:
    """mix_audio.py:14-15."""
    return torch.sqrt(torch.mean(signal ** 2, dim=-1, keepdim=True))


def get_adjusted_rms(clean_rms, snr):
    """mix_audio.py:17-18."""
    return clean_rms / 10 ** (snr / 20)


def _dev_ints(v, device):
    return torch.tensor(v, dtype=torch.int32, device=device)


def mix_batch(clean: torch.Tensor, noise: torch.Tensor, snr_db, noise_start=None, placements=None):
    """Device mixing of B items (se_mix_snr): clean [B, Lc], noise [B, Ln] on the GPU;
    snr_db: B ints; noise_start: B crop starts (used when Ln > Lc); placements: None
    (tiled repeat, noise_repeat=None) or B lists of start indices (noise_repeat given).
    Returns (mix, repeat_noise, scale) as mix_audio.py:95-123 computes them."""
    N.require_device(clean, noise)
    clean, noise = clean.contiguous().float(), noise.contiguous().float()
    B, Lc = clean.shape
    Ln = noise.shape[1]
    if noise.shape[0] != B:
        raise ValueError("sehip mix_batch: one noise clip per clean item")
    dev = clean.device
    starts = _dev_ints(list(noise_start) if noise_start is not None else [0] * B, dev)
    snr = _dev_ints([int(s) for s in snr_db], dev)
    if placements is None:
        nplace, R, place = _dev_ints([-1] * B, dev), 0, None
    else:
        R = max(1, max(len(p) for p in placements))
        flat = [p[r] if r < len(p) else 0 for p in placements for r in range(R)]
        place, nplace = _dev_ints(flat, dev), _dev_ints([len(p) for p in placements], dev)
    mix, rep = torch.empty_like(clean), torch.empty_like(clean)
    scale = torch.empty(B, device=dev, dtype=torch.float32)
    N.check(N.lib().se_mix_snr(clean.data_ptr(), noise.data_ptr(), B, Lc, Ln, starts.data_ptr(), snr.data_ptr(),
                               N.ptr(place), nplace.data_ptr(), R, mix.data_ptr(), rep.data_ptr(),
                               scale.data_ptr(), N.stream_of(clean)), "se_mix_snr")
    return mix, rep, scale


def resample_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """Host table of the band-limited resampler that mix_audio.py:71-77 applies
    (torchaudio.transforms.Resample's default sinc_interp_hann): rates divided by
    their gcd, cut-off min(orig, new) * rolloff, per output phase a Hann-windowed
    sinc over K = 2 width + orig input taps. Returns (kern [new, K] fp32, width,
    orig', new')."""
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float32)[None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float32)[:, None] / new + idx
    t = (t * base).clamp(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    kern = torch.where(t == 0, torch.tensor(1.0), t.sin() / t) * window * (base / orig)
    return kern.contiguous(), width, orig, new


_RESAMPLE_TABLES: dict = {}


def resample(waveform: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """[..., L] on the GPU resampled from orig_freq to new_freq (se_resample), with
    torchaudio.functional.resample's length ceil(new * L / orig)."""
    if int(orig_freq) == int(new_freq):
        return waveform
    N.require_device(waveform)
    key = (int(orig_freq), int(new_freq), str(waveform.device))
    if key not in _RESAMPLE_TABLES:
        kern, width, o, n = resample_kernel(orig_freq, new_freq)
        _RESAMPLE_TABLES[key] = (kern.to(waveform.device), width, o, n)
    kern, width, o, n = _RESAMPLE_TABLES[key]
    x = waveform.reshape(-1, waveform.shape[-1]).contiguous()
    rows, L = x.shape
    lout = math.ceil(n * L / o)
    out = torch.empty(rows, lout, device=x.device, dtype=torch.float32)
    N.check(N.lib().se_resample(x.data_ptr(), rows, L, o, n, kern.data_ptr(), kern.shape[1], width, out.data_ptr(),
                                lout, N.stream_of(x)), "se_resample")
    return out.reshape(waveform.shape[:-1] + (lout,))


def _as_audio(src, sample_rate, device):
    """A path (PCM16 wav, read with its own rate) or a [channels, samples] / [samples]
    tensor (at `sample_rate`), as a [channels, samples] fp32 tensor on the device."""
    if isinstance(src, (str, os.PathLike)):
        return load_wav(src, device=device)
    t = src[None] if src.dim() == 1 else src
    return t.to(device=device, dtype=torch.float32), sample_rate


def get_noisy_data(clean_audio_path, noise_audio_path, mix_output_path="synth/mix/",
                   clean_output_path="synth/clean/", noise_output_path="synth/noise/", mix_sample_rate=16000,
                   clean_sample_rate=None, noise_sample_rate=None, noise_repeat=None, k=100, save=False, *,
                   rng=None, device="cuda"):
    """mix_audio.py:20-149 with the per-sample work on the GPU: the same arguments,
    defaults and return value (clean_amp, noise_amp, outputs), outputs holding the
    reference's keys 'mixed_output', 'adjusted_noise', 'repeat_noise',
    'noise_indices', 'snr' (k entries each). Inputs are paths (16-bit PCM wav;
    torchaudio.load reads more formats) or tensors (channels x samples, or 1-D;
    their rate is clean/noise_sample_rate, default mix_sample_rate). Stereo is
    averaged to mono (:65-69), other rates resampled to mix_sample_rate (:71-77,
    se_resample), then k mixes at random integer SNRs in [-20, 20] are drawn with
    `rng` (a random.Random, or the module `random` as the reference) in the
    reference's order and mixed on the device (se_mix_snr). save=True writes
    <clean>_<noise>_{mix,clean,noise}_<i>.wav as PCM16 into the three output
    directories (:133-138)."""
    rng = rng or _random
    c, csr = _as_audio(clean_audio_path, clean_sample_rate or mix_sample_rate, device)
    n, nsr = _as_audio(noise_audio_path, noise_sample_rate or mix_sample_rate, device)
    if c.shape[0] > 1:
        c = c.mean(dim=0, keepdim=True)
    if n.shape[0] > 1:
        n = n.mean(dim=0, keepdim=True)
    c = resample(c, csr, mix_sample_rate)
    n = resample(n, nsr, mix_sample_rate)
    Lc, Ln = c.shape[1], n.shape[1]
    Lnp = min(Ln, Lc)
    starts, snrs, places, indices = [], [], [], []
    for _ in range(k):                                   # :87-121, same draw order
        starts.append(rng.randint(0, Ln - Lc) if Ln > Lc else 0)
        snrs.append(rng.randint(-20, 20))
        max_repeat = Lc // Lnp
        if noise_repeat is not None:
            p = [rng.randint(0, Lc - Lnp) for _ in range(min(noise_repeat, max_repeat))]
            places.append(p)
            indices.append([[s, s + Lnp] for s in p])
        else:
            indices.append([[i, i + Lnp] for i in range(0, max_repeat * Lnp, Lnp)])
    if k > 0:
        mix, rep, _ = mix_batch(c.expand(k, Lc), n.expand(k, Ln), snrs, starts,
                                places if noise_repeat is not None else None)
    else:
        mix = rep = c.new_empty(0, Lc)
    outputs = {"mixed_output": list(mix.unsqueeze(1).unbind(0)), "adjusted_noise": [n] * k,
               "repeat_noise": list(rep.unsqueeze(1).unbind(0)), "noise_indices": indices, "snr": snrs}
    if save:
        stem = lambda p: os.path.splitext(os.path.basename(str(p)))[0] if isinstance(p, (str, os.PathLike)) else "audio"
        name = stem(clean_audio_path) + "_" + stem(noise_audio_path)
        for d in (mix_output_path, clean_output_path, noise_output_path):
            os.makedirs(d, exist_ok=True)
        for i in range(k):
            save_wav(os.path.join(mix_output_path, f"{name}_mix_{i}.wav"), outputs["mixed_output"][i], mix_sample_rate)
            save_wav(os.path.join(clean_output_path, f"{name}_clean_{i}.wav"), c, mix_sample_rate)
            save_wav(os.path.join(noise_output_path, f"{name}_noise_{i}.wav"), outputs["repeat_noise"][i],
                     mix_sample_rate)
    return c, n, outputs


class AudioSpliter:
    """audio_dataloader.py:8-50: drop items shorter than least_samples, zero-pad
    shorter than chunk_size, else a random chunk (the same start for mix and refs).
    `plan` makes the host decisions in the reference's order; `collate` applies
    them to a ragged batch on the device (se_crop_pad) and stacks like
    default_collate: {'mix': [B, 1, chunk], 'ref': [[B, 1, chunk], ...]}."""

    def __init__(self, chunk_size=32000, least_samples=16000, rng=None):
        self.chunk_size, self.least_samples = chunk_size, least_samples
        self.rng = rng or _random

    def plan(self, lengths):
        """[(keep, start)] per item (:32-48)."""
        out = []
        for L in lengths:
            if L < self.least_samples:
                out.append((False, 0))
            elif L < self.chunk_size:
                out.append((True, 0))
            else:
                out.append((True, self.rng.randint(0, L - self.chunk_size)))
        return out

    def collate(self, samples):
        """samples: [{'mix': [1, L_i], 'ref': [[1, L_i], ...]}] on the GPU."""
        plan = self.plan([s["mix"].shape[-1] for s in samples])
        kept = [(s, st) for s, (keep, st) in zip(samples, plan) if keep]
        if not kept:
            return []
        dev = kept[0][0]["mix"].device
        lens = [s["mix"].shape[-1] for s, _ in kept]
        offs = [0]
        for L in lens[:-1]:
            offs.append(offs[-1] + L)
        off_t = torch.tensor(offs, dtype=torch.int64, device=dev)
        len_t, st_t = _dev_ints(lens, dev), _dev_ints([st for _, st in kept], dev)

        def crop(stream):
            src = torch.cat([t.reshape(-1).float() for t in stream]).contiguous()
            N.require_device(src)
            out = torch.empty(len(kept), 1, self.chunk_size, device=dev, dtype=torch.float32)
            N.check(N.lib().se_crop_pad(src.data_ptr(), off_t.data_ptr(), len_t.data_ptr(), st_t.data_ptr(),
                                        len(kept), self.chunk_size, out.data_ptr(), N.stream_of(src)),
                    "se_crop_pad")
            return out

        nref = len(kept[0][0]["ref"])
        return {"mix": crop([s["mix"] for s, _ in kept]),
                "ref": [crop([s["ref"][j] for s, _ in kept]) for j in range(nref)]}


class AudioDataLoader:
    """audio_dataloader.py:52-81: a torch DataLoader over `dataset` (items
    {'mix': [1, L], 'ref': [[1, L], ...]}, as TrainAudioDatasets yields) whose
    workers only gather the ragged items; each batch is then cropped / padded to
    chunk_size and stacked on the device (AudioSpliter.collate, se_crop_pad).
    Items shorter than least_samples are dropped (audio_dataloader.py:32-34).
    Yields {'mix': [B, 1, chunk], 'ref': [[B, 1, chunk], ...]} on `device`;
    len() is the dataset length, as the reference's.
    The chunk-start draws are made in this (main) process with `rng`. The reference
    makes them inside its collate_fn, i.e. in each DataLoader worker's own seeded
    `random` when num_workers > 0, so a seeded run picks the reference's crops only
    with num_workers=0."""

    def __init__(self, dataset, chunk_size=32000, least_samples=16000, device="cuda", rng=None, **kwargs):
        from torch.utils.data import DataLoader
        self.dataset = dataset
        self.batch_size = kwargs["batch_size"]
        self.device = device
        self.spliter = AudioSpliter(chunk_size, least_samples, rng=rng)
        self.data_loader = DataLoader(dataset, collate_fn=list, **kwargs)

    def __iter__(self):
        for items in self.data_loader:
            on_dev = [{"mix": it["mix"].to(self.device, non_blocking=True),
                       "ref": [r.to(self.device, non_blocking=True) for r in it["ref"]]} for it in items]
            batch = self.spliter.collate(on_dev)
            if batch:          # every item shorter than least_samples: nothing to yield
                yield batch

    def __len__(self):
        return len(self.dataset)


def pcm16_to_float(x: torch.Tensor) -> torch.Tensor:
    """int16 samples -> float / 32768 (torchaudio.load's normalisation), on the device."""
    N.require_device(x, dtype=torch.int16)
    x = x.contiguous()
    out = torch.empty(x.shape, device=x.device, dtype=torch.float32)
    N.check(N.lib().se_pcm16_to_float(x.data_ptr(), x.numel(), out.data_ptr(), N.stream_of(x)),
            "se_pcm16_to_float")
    return out


def float_to_pcm16(x: torch.Tensor) -> torch.Tensor:
    """float -> int16 = clamp(rint(x * 32768)) (PCM_S 16-bit save, mix_audio.py:144-146)."""
    N.require_device(x)
    x = x.contiguous().float()
    out = torch.empty(x.shape, device=x.device, dtype=torch.int16)
    N.check(N.lib().se_float_to_pcm16(x.data_ptr(), x.numel(), out.data_ptr(), N.stream_of(x)),
            "se_float_to_pcm16")
    return out


def load_wav(path, device="cuda") -> tuple[torch.Tensor, int]:
    """PCM16 wav -> ([channels, samples] float on the device, sample rate)."""
    with _wave.open(str(path), "rb") as f:
        if f.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM wav is supported")
        ch, sr, n = f.getnchannels(), f.getframerate(), f.getnframes()
        raw = f.readframes(n)
    pcm = torch.frombuffer(bytearray(raw), dtype=torch.int16).view(n, ch).t().contiguous()
    return pcm16_to_float(pcm.to(device)), sr


def save_wav(path, audio: torch.Tensor, sr: int) -> None:
    """[channels, samples] (or [samples]) float on the device -> PCM16 wav."""
    a = audio[None] if audio.dim() == 1 else audio
    pcm = float_to_pcm16(a).cpu().t().contiguous()
    with _wave.open(str(path), "wb") as f:
        f.setnchannels(a.shape[0])
        f.setsampwidth(2)
        f.setframerate(int(sr))
        f.writeframes(pcm.numpy().tobytes())
