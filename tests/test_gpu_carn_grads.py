"""CARN / GCARN training gradients (models/_2104_05267_carn.py) per tensor against an fp64
CPU run of the oracle — with the Linear(512 -> 514) head (carn.py:133, 157-159) on the
hand-written GEMM (sehip.linear), the attention gates / decoder cat / mask / clamp on the
HIP glue passes (sehip.glue), and every conv / BN + PReLU / LSTM on their kernels
("a CARN fp32 gradient check vs fp64 that includes the Linear").

Gate (as DCUNet-20's, tests/test_gpu_variants.py): each tensor's rel-L2 vs fp64 within
max(3x the largest error of the fp32 CPU evaluations (unperturbed, and two 2^-22 relative
input perturbations), 1e-4); the median over tensors within 3x the largest median of
those evaluations. Plus the forward (spec, wav) within the north star's 1e-4."""
import numpy as np
import pytest
import torch

import paramfill
from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _carn_grads(dev, dtype, gate, sehip=False, perturb=0.0, seed=1234):
    from oracle import models as O, train as OT
    noisy, clean = paramfill.structured_pair(1, 8000, seed=43)
    if sehip:
        from sehip import models as M
        from sehip.losses import SI_SNR_loss as loss_fn, pad_or_truncate_wav as pad
        m = (M.GCARN if gate else M.CARN)(320, 160, 512)
    else:
        loss_fn, pad = OT.si_snr_loss, OT.pad_or_truncate_wav
        m = (O.GCARN if gate else O.CARN)(320, 160, 512)
    m = paramfill.fill_(m, seed=77).to(dev).to(dtype).train()
    x = torch.from_numpy(noisy).to(dtype)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=gen, dtype=torch.float64)).to(dtype)
    c = torch.from_numpy(clean).to(dev).to(dtype)
    spec, w = m(x.to(dev))
    loss_fn(pad(w, c), c).backward()
    return ({n: p.grad.detach().double().cpu() for n, p in m.named_parameters()},
            spec.detach().double().cpu(), w.detach().double().cpu())


@pytest.mark.parametrize("gate", [False, True], ids=["carn", "gcarn"])
def test_carn_train_grads_vs_fp64(gate, gpu_device):
    from sehip import linear as LN
    g64, s64, w64 = _carn_grads("cpu", torch.float64, gate)
    evals = [_carn_grads("cpu", torch.float32, gate)[0]] + \
        [_carn_grads("cpu", torch.float32, gate, perturb=2.0 ** -22, seed=1234 + i)[0] for i in range(2)]
    n0 = LN.LINEAR_CALLS[0]
    gh, sh, wh = _carn_grads("cuda", torch.float32, gate, sehip=True)
    assert LN.LINEAR_CALLS[0] == n0 + 1          # the head ran on se_gemm
    assert sorted(gh) == sorted(g64) and "linear.weight" in gh and "linear.bias" in gh
    es, ew = rel_l2(sh.numpy(), s64.numpy()), rel_l2(wh.numpy(), w64.numpy())
    assert es < 1e-4 and ew < 1e-4, (es, ew)
    rel = lambda g, n: (g[n] - g64[n]).norm().item() / (g64[n].norm().item() + 1e-30)
    rows = [(rel(gh, n), max(rel(q, n) for q in evals), n) for n in g64]
    bad = [r for r in rows if r[0] > max(3 * r[1], 1e-4)]
    med_h = np.median([r[0] for r in rows])
    med_o = max(np.median([rel(q, n) for n in g64]) for q in evals)
    lin = [r for r in rows if r[2].startswith("linear.")]
    print(f"{'gcarn' if gate else 'carn'} grads vs fp64: median hip {med_h:.2e}, fp32 evaluations up to "
          f"{med_o:.2e}; head {[(f'{r[0]:.1e}', r[2]) for r in lin]}; fwd spec {es:.1e} wav {ew:.1e}")
    assert not bad, sorted(bad, key=lambda r: -r[0])[:5]
    assert med_h < 3 * med_o, (med_h, med_o)
