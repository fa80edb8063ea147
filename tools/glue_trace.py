"""Where the ATen glue of configs 2/3 comes from: one DCUNet-16 bf16 forward and one
DCCRN-CL bf16 train step under torch.profiler (with_stack), listing every aten op that
launches a GPU kernel outside sehip's own library, grouped by the innermost sehip frames.

Usage: python tools/glue_trace.py [--configs 2,3] [--storage bf16]"""
import argparse, collections, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import traceback
import torch
from torch.utils._python_dispatch import TorchDispatchMode

GLUE = ("aten::cat", "aten::copy_", "aten::_to_copy", "aten::add", "aten::add_", "aten::mul", "aten::fill_",
        "aten::zero_", "aten::constant_pad_nd", "aten::clone", "aten::contiguous", "aten::sub", "aten::div",
        "aten::sum", "aten::neg", "aten::stack", "aten::index", "aten::slice_scatter", "aten::maximum")


class _Glue(TorchDispatchMode):
    """Counts every aten op that runs on a GPU tensor, keyed by op, first input shape
    and the innermost repository frames that issued it."""

    def __init__(self):
        super().__init__()
        self.agg = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        if name not in ("view", "_unsafe_view", "empty", "empty_like", "empty_strided", "as_strided", "t",
                        "detach", "alias", "expand", "permute", "select", "slice", "unsqueeze", "squeeze",
                        "transpose", "reshape", "split", "chunk", "unbind", "lift_fresh", "_to_copy_noop"):
            t0 = next((a for a in args if isinstance(a, torch.Tensor)), None)
            if t0 is None and args and isinstance(args[0], (list, tuple)) and args[0] and isinstance(args[0][0], torch.Tensor):
                t0 = args[0][0]
            if t0 is not None and t0.is_cuda:
                st = [f for f in traceback.extract_stack()[:-1]
                      if ("sehip" in f.filename or "tools" in f.filename) and "glue_trace" not in f.filename]
                fr = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[::-1][:3])
                self.agg[(name, str(tuple(t0.shape))[:40], str(t0.dtype)[6:], fr)] += 1
        return out


def run(name, fn):
    fn()
    torch.cuda.synchronize()
    with _Glue() as g:
        fn()
        torch.cuda.synchronize()
    print(f"== {name}")
    for (n, s, dt, fr), c in sorted(g.agg.items(), key=lambda kv: -kv[1]):
        print(f"{c:4d}  {n:18s} {s:40s} {dt:9s} {fr}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3")
    ap.add_argument("--storage", default="bf16")
    a = ap.parse_args()
    from sehip import functional as F, models as M
    from sehip.data import synthetic_pairs
    from sehip.train import make_optimizer, train_step
    dev = torch.device("cuda")
    calls = collections.Counter()

    def wrap(mod, name):
        fn = getattr(mod, name)

        def w(*a, **k):
            st = [f for f in traceback.extract_stack()[:-1] if "sehip" in f.filename]
            shp = [tuple(t.shape) for t in a if isinstance(t, torch.Tensor)]
            calls[(name, str(shp), " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[::-1][:3]))] += 1
            return fn(*a, **k)
        setattr(mod, name, w)
    wrap(F, "_join_raw")
    wrap(F, "complex_join")
    import atexit
    atexit.register(lambda: [print(f"{c:4d}  {k}") for k, c in calls.items()])
    sdt = torch.bfloat16 if a.storage == "bf16" else torch.float32
    F.set_conv_math("bf16")
    if "2" in a.configs:
        m = M.DCUNet("dcunet16", 512, 128, 512).to(dev).eval().to(sdt)
        x, _ = synthetic_pairs(16, 64000, seed=5, device=dev)
        x = x.to(sdt)
        with torch.no_grad():
            run("config 2 DCUNet-16 forward", lambda: m(x))
    if "3" in a.configs:
        m = M.DCCRN("dccrn-CL", 400, 100, 512).to(dev).train().to(sdt)
        opt = make_optimizer(m)
        x, c = synthetic_pairs(64, 64000, seed=6, device=dev)
        x, c = x.to(sdt), c.to(sdt)
        run("config 3 DCCRN-CL train step", lambda: train_step(m, opt, x, c))


if __name__ == "__main__":
    main()
