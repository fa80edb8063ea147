"""Long-form inference in chunks (BASELINE.json config 5: CARN on 30 s @ 48 kHz).

The reference enhances a whole utterance in one forward (carn.py:135-172); a
30 s @ 48 kHz input is one [1, 1,440,000] sequence whose 9002-frame LSTM
recurrence is the latency floor. Here the waveform is cut into fixed chunks of
`chunk` samples, consecutive chunks overlapping by `overlap` samples, the
chunks run as ONE batch (one launch per op for the whole utterance), and the
enhanced chunks are overlap-added with a linear cross-fade over each overlap
(sum of the two fade weights = 1), then trimmed to the input length. The last
chunk is zero-padded. The same procedure, on the oracle model, is
oracle/longform.py. On the GPU the split and the cross-fade overlap-add are one HIP
pass each (glue.chunk_split / glue.chunk_overlap_add, csrc/glue.hip); the torch
forms below are the same arithmetic for host tensors.
"""
from __future__ import annotations

import torch


def chunk_plan(length: int, chunk: int, overlap: int):
    """Start sample of every chunk: hop = chunk - overlap; enough chunks to cover length."""
    if chunk <= 0 or not 0 <= overlap < chunk:
        raise ValueError("need chunk > 0 and 0 <= overlap < chunk")
    hop = chunk - overlap
    n = max(1, -(-max(length - overlap, 1) // hop))
    return [i * hop for i in range(n)]


def split_chunks(wav: torch.Tensor, chunk: int, overlap: int) -> torch.Tensor:
    """[L] or [1, L] -> [n, chunk] (zero-padded at the end)."""
    x = wav.reshape(-1)
    starts = chunk_plan(x.shape[0], chunk, overlap)
    if x.is_cuda:
        from . import glue
        return glue.chunk_split(x, chunk, starts)
    total = starts[-1] + chunk
    xp = torch.nn.functional.pad(x, (0, total - x.shape[0]))
    return xp.unfold(0, chunk, chunk - overlap)[: len(starts)].contiguous()


def overlap_add(chunks: torch.Tensor, length: int, overlap: int) -> torch.Tensor:
    """[n, chunk] -> [length]: linear cross-fade over each overlap."""
    n, chunk = chunks.shape
    hop = chunk - overlap
    if chunks.is_cuda:
        from . import glue
        return glue.chunk_overlap_add(chunks, chunk, overlap, length)
    w = torch.ones(chunk, device=chunks.device, dtype=chunks.dtype)
    if overlap:
        ramp = (torch.arange(overlap, device=chunks.device, dtype=torch.float32) + 0.5) / overlap
        w_in, w_out = ramp.to(chunks.dtype), (1 - ramp).to(chunks.dtype)
    out = torch.zeros(hop * (n - 1) + chunk, device=chunks.device, dtype=chunks.dtype)
    for i in range(n):
        c = chunks[i] * w
        if overlap and i > 0:
            c[:overlap] = chunks[i, :overlap] * w_in
        if overlap and i < n - 1:
            c[chunk - overlap:] = chunks[i, chunk - overlap:] * w_out
        out[i * hop:i * hop + chunk] += c
    return out[:length]


@torch.no_grad()
def enhance_chunked(model, wav: torch.Tensor, chunk: int, overlap: int = 0, max_batch: int | None = None):
    """Enhance a long waveform [L] / [1, L] with `model` (forward(x) -> (spec, wav))
    in chunks; returns the enhanced waveform [1, L]. max_batch bounds how many
    chunks run per forward (None = all at once)."""
    length = wav.reshape(-1).shape[0]
    chunks = split_chunks(wav, chunk, overlap)
    outs = []
    step = max_batch or chunks.shape[0]
    for i in range(0, chunks.shape[0], step):
        _, y = model(chunks[i:i + step])
        outs.append(y.reshape(y.shape[0], -1))
    if wav.is_cuda and len(outs) == 1:
        # the rows read up to their own width (a shorter iSTFT output counts as zero-padded:
        # DCCRN) in the overlap-add pass itself
        from . import glue
        return glue.chunk_overlap_add(outs[0], chunk, overlap, length)[None]
    outs = [torch.nn.functional.pad(y, (0, chunk - y.shape[1])) if y.shape[1] < chunk else y[:, :chunk]
            for y in outs]                           # models whose iSTFT shortens (DCCRN)
    return overlap_add(torch.cat(outs), length, overlap)[None]
