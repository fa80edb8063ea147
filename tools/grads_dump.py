"""Dump the FRCRN train-step parameter gradients (HIP path, default conv math)
to a file, or compare two dumps bit for bit. Used to check that a kernel
variant selected by an environment knob is bit-identical to the default:
  SEHIP_X=1 python tools/grads_dump.py dump a.pt && python tools/grads_dump.py dump b.pt
  python tools/grads_dump.py cmp a.pt b.pt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def dump(path, batch=4, seconds=1):
    import paramfill
    from sehip.losses import SI_SNR_loss
    from sehip.models import FRCRN
    m = paramfill.fill_(FRCRN(), seed=9).cuda().train()
    noisy, clean = (torch.from_numpy(t).cuda() for t in paramfill.structured_pair(batch, 16000 * seconds, seed=60))
    _, wav = m(noisy)
    SI_SNR_loss(wav, clean).backward()
    torch.cuda.synchronize()
    torch.save({n: p.grad.detach().cpu() for n, p in m.named_parameters()}, path)


def cmp(a, b):
    ga, gb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [n for n in ga if not torch.equal(ga[n], gb[n])]
    worst = max(((ga[n] - gb[n]).norm() / (ga[n].norm() + 1e-30)).item() for n in ga)
    print(f"{len(bad)} of {len(ga)} gradients differ; worst rel-L2 {worst:.2e}; first: {bad[:6]}")
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
