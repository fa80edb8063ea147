"""Oracle twin of sehip/longform.py (test infrastructure only): the same chunk
plan, zero padding and linear cross-fade overlap-add around the oracle model,
on the CPU. The reference has no chunked mode (carn.py:135-172 enhances the
whole input); BASELINE config 5 names 30 s @ 48 kHz "chunks", so the chunking
itself is this build's definition and the oracle checks the model math inside
it."""
from __future__ import annotations

import torch


def enhance_chunked(model, wav, chunk, overlap=0):
    x = wav.reshape(-1)
    L = x.shape[0]
    hop = chunk - overlap
    n = max(1, -(-max(L - overlap, 1) // hop))
    xp = torch.nn.functional.pad(x, (0, (n - 1) * hop + chunk - L))
    out = torch.zeros((n - 1) * hop + chunk, dtype=x.dtype)
    for i in range(n):
        with torch.no_grad():
            _, y = model(xp[i * hop:i * hop + chunk][None])
        y = torch.nn.functional.pad(y.reshape(-1), (0, max(0, chunk - y.numel())))[:chunk]
        w = torch.ones(chunk, dtype=x.dtype)
        if overlap:
            ramp = ((torch.arange(overlap, dtype=torch.float32) + 0.5) / overlap).to(x.dtype)
            if i > 0:
                w[:overlap] = ramp
            if i < n - 1:
                w[chunk - overlap:] = 1 - ramp
        out[i * hop:i * hop + chunk] += y * w
    return out[:L][None]
