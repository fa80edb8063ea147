"""BASELINE config 5: CARN (_2104_05267_carn) fp16, long-form input in chunks.

* fp16 storage (model.half(), as the reference's low-precision run): the
  enhanced output against the fp32 golden, gated by the oracle's own fp16
  drift on the same parameters and input (CARN fp16 2 s
  9.2e-4 from fp32), like the bf16 configs in test_gpu_models.py.
* the chunked long-form path (sehip/longform.py: fixed chunks as one batch,
  linear cross-fade overlap-add) against oracle/longform.py around the oracle
  CARN, fp32 at the north-star 1e-4 bar and fp16 within the oracle's drift.
"""
import pytest
import torch

from conftest import golden, rel_l2
import paramfill

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _carn(mod, gate):
    return (mod.GCARN if gate else mod.CARN)(320, 160, 512)


@pytest.mark.parametrize("gate,name,seed", [(False, "carn", 23), (True, "gcarn", 24)])
def test_carn_fp16_within_oracle_fp16_drift(gate, name, seed, gpu_device):
    from sehip import models as M
    from oracle import models as O
    g = golden(f"model_{name}")
    x = torch.from_numpy(g["x"])
    # train mode: with random-init weights the eval-mode running statistics (mean 0,
    # var 1) let the activations outgrow fp16 (oracle and ours both drift ~0.5 there);
    # batch statistics keep them in range, as a trained model's statistics would
    mo = paramfill.fill_(_carn(O, gate), seed=seed).half().train()
    with torch.no_grad():
        so, wo = mo(x.half())
    drift = max(rel_l2(so.float().numpy(), g["spec_train"]), rel_l2(wo.float().numpy(), g["wav_train"]))
    assert drift < 1e-2, drift   # a meaningful fp16 gate
    m = paramfill.fill_(_carn(M, gate), seed=seed).cuda().half().train()
    assert m.stft._tw.dtype == torch.float32 and m.istft._win.dtype == torch.float32   # kernel tables stay fp32
    with torch.no_grad():
        s, w = m(x.cuda().half())
    assert s.dtype == torch.float16 and w.dtype == torch.float16
    es = rel_l2(s.float().cpu().numpy(), g["spec_train"])
    ew = rel_l2(w.float().cpu().numpy(), g["wav_train"])
    print(f"{name} fp16: ours spec {es:.2e} wav {ew:.2e}; oracle fp16 drift {drift:.2e}")
    assert max(es, ew) < max(3 * drift, 1e-3), (es, ew, drift)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_carn_chunked_longform_vs_oracle(dtype, gpu_device):
    """3 s @ 48 kHz in 1 s chunks overlapping by 0.1 s (4 chunks, one batch)."""
    from sehip import models as M, longform as L
    from oracle import models as O, longform as OL
    sr, chunk, overlap = 48000, 48000, 4800
    noisy, _ = paramfill.structured_pair(1, 3 * sr, seed=31)
    x = torch.from_numpy(noisy)[0]
    mo = paramfill.fill_(O.CARN(320, 160, 512), seed=32).eval()
    ref32 = OL.enhance_chunked(mo, x, chunk, overlap)
    m = paramfill.fill_(M.CARN(320, 160, 512), seed=32).cuda().eval().to(dtype)
    got = L.enhance_chunked(m, x.cuda().to(dtype), chunk, overlap)
    assert got.shape == (1, x.shape[0]) and got.dtype == dtype
    e = rel_l2(got.float().cpu().numpy(), ref32.numpy())
    if dtype == torch.float32:
        assert e < TOL, e
    else:
        ref16 = OL.enhance_chunked(mo.half(), x.half(), chunk, overlap)
        drift = rel_l2(ref16.float().numpy(), ref32.numpy())
        print(f"chunked fp16: ours {e:.2e}, oracle fp16 drift {drift:.2e}")
        assert e < max(3 * drift, 1e-3), (e, drift)


@pytest.mark.timeout(600)
def test_carn_config5_full_length_vs_oracle(gpu_device):
    """BASELINE config 5 at its full size: one 30 s @ 48 kHz utterance
    ([1, 1,440,000]) through CARN in 4 s chunks overlapping 50 ms (8 chunks, one
    batch; tools/bench_configs.py's plan). fp32 against oracle/longform.py at the
    north-star 1e-4; fp16 storage (model.half()) against the same fp32 oracle
    within 3x the oracle's own fp16 drift, measured on the first two chunks (the
    CPU's fp16 convolutions take ~15 s per chunk)."""
    from sehip import models as M, longform as L
    from oracle import models as O, longform as OL
    sr, chunk, overlap = 48000, 4 * 48000, 48000 // 20
    noisy, _ = paramfill.structured_pair(1, 30 * sr, sr=sr, seed=35)
    x = torch.from_numpy(noisy)[0]
    mo = paramfill.fill_(O.CARN(320, 160, 512), seed=36).eval()
    ref32 = OL.enhance_chunked(mo, x, chunk, overlap)
    m = paramfill.fill_(M.CARN(320, 160, 512), seed=36).cuda().eval()
    got = L.enhance_chunked(m, x.cuda(), chunk, overlap)
    assert got.shape == (1, 30 * sr)
    e32 = rel_l2(got.cpu().numpy(), ref32.numpy())
    got16 = L.enhance_chunked(m.half(), x.cuda().half(), chunk, overlap)
    e16 = rel_l2(got16.float().cpu().numpy(), ref32.numpy())
    head = 2 * chunk - overlap                   # the first two chunks' span
    ref_head32 = OL.enhance_chunked(mo, x[:head], chunk, overlap)
    ref_head16 = OL.enhance_chunked(mo.half(), x[:head].half(), chunk, overlap)
    drift = rel_l2(ref_head16.float().numpy(), ref_head32.numpy())
    print(f"config 5, 30 s @ 48 kHz chunked: fp32 {e32:.2e}; fp16 {e16:.2e} (oracle fp16 drift {drift:.2e})")
    assert e32 < TOL, e32
    assert e16 < max(3 * drift, 1e-3), (e16, drift)
