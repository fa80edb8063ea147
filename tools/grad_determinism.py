"""Which FRCRN gradients vary from run to run: R forward + SI-SNR + backward passes on the
same parameters and batch, every parameter .grad (and the loss) compared bit for bit with
the first run's; per mode (inline: SEHIP_OVERLAP=0, full: side streams on) the names of the
tensors that ever differ, with the largest difference seen.

Usage: python tools/grad_determinism.py [--runs 30] [--batch 2] [--seconds 1] [--modes inline,full]"""
import argparse, collections, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--modes", default="inline,full")
    a = ap.parse_args()
    import paramfill
    from sehip import models as M, train as T, losses as Lo
    from sehip import functional as F
    noisy, clean = paramfill.structured_pair(a.batch, int(16000 * a.seconds), seed=8)
    x, c = torch.from_numpy(noisy).cuda(), torch.from_numpy(clean).cuda()
    m = paramfill.fill_(M.FRCRN(), seed=9).cuda().train()
    names = [n for n, _ in m.named_parameters()]
    for mode in a.modes.split(","):
        os.environ["SEHIP_OVERLAP"] = "0" if mode == "inline" else "1"
        ref, bad = None, collections.defaultdict(float)
        nbad = 0
        for r in range(a.runs):
            for p in m.parameters():
                p.grad = None
            _, wav = m(x)
            loss = Lo.si_snr_loss_aligned(wav, c)
            with F.deferred_weight_grads(T._defer_ok(m)):
                loss.backward()
            T.finish_grads(m)
            torch.cuda.synchronize()
            res = [loss.detach().clone()] + [p.grad.detach().clone() for p in m.parameters()]
            if ref is None:
                ref = res
                continue
            diff = False
            for i, (u, v) in enumerate(zip(ref, res)):
                if not torch.equal(u, v):
                    diff = True
                    k = "loss" if i == 0 else names[i - 1]
                    bad[k] = max(bad[k], (u - v).abs().max().item())
            nbad += diff
        print(f"{mode}: {nbad} of {a.runs - 1} runs differ from run 0", flush=True)
        for k, v in sorted(bad.items(), key=lambda kv: -kv[1])[:40]:
            print(f"   {v:.3e}  {k}", flush=True)


if __name__ == "__main__":
    main()
