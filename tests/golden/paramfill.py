"""Name-keyed deterministic parameter fill.

Golden fixtures store inputs, outputs and this *recipe* instead of 7.7 MB of
weights: every state_dict entry is filled from
``np.random.RandomState(crc32(name) ^ seed)`` with a distribution chosen by
the entry's leaf name, so the reference model (in gen_golden.py), the oracle
restatement and the HIP path all receive bit-identical weights without
sharing any code but this file. Pure numpy + torch; no reference import.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

# deterministic DSP buffers recomputed by every implementation (conv_stft.py:40,80-82)
_SKIP_SUFFIX = ("num_batches_tracked",)
_SKIP_PREFIX_LEAVES = ("stft.weight", "istft.weight", "istft.window", "istft.enframe")


def _draw(name: str, shape: tuple, seed: int) -> np.ndarray | None:
    rs = np.random.RandomState((zlib.crc32(name.encode()) ^ seed) & 0xFFFFFFFF)
    leaf = name.rsplit(".", 1)[-1]
    n = int(np.prod(shape)) if shape else 1
    if leaf in ("Wrr", "Wii"):
        v = 1.0 + 0.1 * rs.uniform(-1, 1, n)
    elif leaf == "Wri":
        v = rs.uniform(-0.4, 0.4, n)          # keeps W positive definite
    elif leaf in ("Br", "Bi"):
        v = 0.05 * rs.standard_normal(n)
    elif leaf in ("RMr", "RMi", "running_mean"):
        v = 0.1 * rs.standard_normal(n)
    elif leaf in ("RVrr", "RVii", "running_var"):
        v = 1.0 + 0.2 * rs.uniform(0, 1, n)
    elif leaf == "RVri":
        v = 0.1 * rs.uniform(-1, 1, n)
    elif "lstm" in name and leaf.startswith("weight"):
        hidden = shape[0] // 4
        b = 1.0 / math.sqrt(hidden)
        v = rs.uniform(-b, b, n)
    elif leaf.startswith("bias"):
        v = 0.05 * rs.standard_normal(n)
    elif leaf == "weight" and len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = rs.standard_normal(n) * math.sqrt(2.0 / fan_in)
    elif leaf == "weight" and len(shape) == 1:
        # nn.BatchNorm2d.weight or nn.PReLU.weight
        v = (0.25 if shape[0] == 1 else 1.0) + 0.05 * rs.uniform(-1, 1, n)
    else:
        v = 0.1 * rs.standard_normal(n)
    return v.reshape(shape)


@torch.no_grad()
def fill_(model: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    for name, t in model.state_dict().items():
        if name.endswith(_SKIP_SUFFIX) or any(name.endswith(s) for s in _SKIP_PREFIX_LEAVES):
            continue
        if not t.is_floating_point():
            continue
        v = _draw(name, tuple(t.shape), seed)
        t.copy_(torch.from_numpy(v).to(t.dtype))
    return model


def structured_pair(batch: int, length: int, sr: int = 16000, seed: int = 0):
    """Structured noisy/clean pair (SURVEY.md §8c 'Gradient parity'): an AM
    harmonic tone + light noise as clean, noisy = clean + 0.1 N(0,1)."""
    rs = np.random.RandomState(seed)
    t = np.arange(length) / sr
    clean = np.zeros((batch, length))
    for b in range(batch):
        f0 = 150.0 + 40.0 * b
        env = 1.0 + 0.5 * np.sin(2 * np.pi * 3.0 * t + b)
        clean[b] = 0.3 * np.sin(2 * np.pi * f0 * t) * env + 0.1 * np.sin(2 * np.pi * 2 * f0 * t)
    clean += 0.05 * rs.standard_normal(clean.shape)
    noisy = clean + 0.1 * rs.standard_normal(clean.shape)
    return noisy.astype(np.float32), clean.astype(np.float32)
