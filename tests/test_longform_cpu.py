"""CPU: the chunk plan covers the input, and split + cross-fade overlap-add is
the identity (the fade weights sum to 1 in every overlap)."""
import pytest
import torch


@pytest.mark.parametrize("L,chunk,overlap", [(10007, 3000, 0), (10007, 3000, 500), (1440000, 192000, 4800),
                                             (100, 3000, 200), (6000, 3000, 0)])
def test_split_overlap_add_identity(L, chunk, overlap):
    from sehip import longform as LF
    x = torch.randn(L)
    starts = LF.chunk_plan(L, chunk, overlap)
    assert starts[0] == 0 and starts[-1] + chunk >= L
    c = LF.split_chunks(x, chunk, overlap)
    assert c.shape == (len(starts), chunk)
    assert torch.allclose(LF.overlap_add(c, L, overlap), x, atol=1e-6)
