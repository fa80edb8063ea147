"""CPU: the reference trainer's initialize_params (utils.py:47-84, called by
train.py:38) reaches the same modules of sehip's drop-in models as of the
reference formulation (the oracle) — every real_conv / imag_conv weight
holder of the fused complex convs included — and leaves ComplexBatchNorm2d's
parameters alone (it is no nn.BatchNorm2d), as in the reference."""
import pytest
import torch

from oracle import models as O
from oracle.train import initialize_params

MODELS = [("FRCRN", {}), ("DCCRN", {}), ("DCUNet", {"config": "dcunet16"}), ("CARN", {}), ("GCARN", {}),
          ("CRN", {})]


@pytest.mark.parametrize("name,kw", MODELS, ids=[m[0] for m in MODELS])
def test_initialize_params_visits_the_same_modules(name, kw):
    from sehip import models as M
    torch.manual_seed(0)
    ref = getattr(O, name)(**kw)
    torch.manual_seed(0)
    mod = getattr(M, name)(**kw)
    visited_ref = initialize_params(ref)
    visited = initialize_params(mod)
    assert visited == visited_ref
    if name in ("FRCRN", "DCCRN", "DCUNet"):
        assert any(v.endswith("real_conv") for v in visited) and any(v.endswith("imag_conv") for v in visited)


def test_initialize_params_reinitialises_fused_conv_holders():
    """Every real_conv / imag_conv weight of sehip.FRCRN is redrawn with the
    kaiming-normal std sqrt(2 / fan_in); ComplexBatchNorm2d's W/B and running
    statistics are untouched."""
    from sehip import models as M
    from sehip.complex_nn import ComplexBatchNorm2d
    torch.manual_seed(1)
    m = M.FRCRN()
    before = {k: v.clone() for k, v in m.state_dict().items()}
    initialize_params(m)
    after = m.state_dict()
    convs = [n for n, mod in m.named_modules() if n.endswith(("real_conv", "imag_conv"))]
    assert len(convs) == 2 * (6 + 6 + 6)   # encoder, decoder, CCBAM spatial convs
    for n in convs:
        w = after[n + ".weight"]
        assert not torch.equal(w, before[n + ".weight"]), n
        fan_in = w.shape[1] * w[0, 0].numel()
        std = (2.0 / fan_in) ** 0.5
        assert abs(w.std().item() / std - 1) < 0.25 or w.numel() < 64, (n, w.std().item(), std)
    for n, mod in m.named_modules():
        if isinstance(mod, ComplexBatchNorm2d):
            for p in ("Wrr", "Wri", "Wii", "Br", "Bi", "RMr", "RMi", "RVrr", "RVri", "RVii"):
                assert torch.equal(after[f"{n}.{p}"], before[f"{n}.{p}"]), (n, p)
