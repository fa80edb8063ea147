"""Which Python lines still launch ATen / hipBLASLt kernels in a config's step.

Runs one warm step of a BASELINE config under torch.profiler (CPU + GPU
activity, Python stacks) and prints, per (kernel family, innermost sehip /
model frame), the launch count: every GPU kernel whose name marks it as
PyTorch's own (at::native, Cijk_ hipBLASLt, rocclr copies) is attributed to
the Python line that issued it. Diagnostic only.

  python tools/aten_sources.py --config 3|5|4 [--storage bf16|fp16|fp32]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import torch


def _family(name: str) -> str | None:
    if "at::native" in name or name.startswith("void at::"):
        return "aten:" + name.split("<")[0].replace("void ", "")[:60] + ("<" + name.split("<")[1][:70]
                                                                        if "<" in name else "")
    if name.startswith("Cijk_"):
        return "hipblaslt:Cijk"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--storage", default=None)
    a = ap.parse_args()
    from sehip import functional as F, models as M, longform as L
    from sehip.data import synthetic_pairs
    from sehip.train import make_optimizer, train_step
    dev = torch.device("cuda")
    if a.config == 3:
        st = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.storage or "bf16"]
        F.set_conv_math("bf16")
        m = M.DCCRN("dccrn-CL", 400, 100, 512).to(dev).train().to(st)
        opt = make_optimizer(m)
        x, c = synthetic_pairs(8, 64000, seed=6, device=dev)
        x, c = x.to(st), c.to(st)
        fn = lambda: train_step(m, opt, x, c)
    elif a.config == 5:
        st = {"fp16": torch.float16, "fp32": torch.float32}[a.storage or "fp16"]
        m = M.CARN(320, 160, 512).to(dev).eval().to(st)
        x, _ = synthetic_pairs(1, 48000 * 30, sr=48000, seed=7, device=dev)
        x = x.to(st)
        fn = lambda: L.enhance_chunked(m, x, 4 * 48000, 48000 // 20)
    elif a.config == 2:
        st = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.storage or "bf16"]
        F.set_conv_math("bf16")
        m = M.DCUNet("dcunet16", 512, 128, 512).to(dev).eval().to(st)
        x, _ = synthetic_pairs(4, 64000, seed=5, device=dev)
        x = x.to(st)
        fn = lambda: m(x)
    else:
        m = M.FRCRN().to(dev).train()
        opt = make_optimizer(m)
        x, c = synthetic_pairs(4, 64000, seed=6, device=dev)
        fn = lambda: train_step(m, opt, x, c)
    ctx = torch.no_grad() if a.config in (2, 5) else torch.enable_grad()
    with ctx:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
            fn()
            torch.cuda.synchronize()
    counts = collections.Counter()
    total = collections.Counter()
    for ev in prof.events():
        kern = [k for k in getattr(ev, "kernels", [])]
        if not kern:
            continue
        fams = [f for f in (_family(k.name) for k in kern) if f]
        if not fams:
            continue
        e, stack = ev, []
        while e is not None and not stack:   # the nearest ancestor op that recorded Python frames
            stack = [s for s in (e.stack or [])]
            e = e.cpu_parent
        frames = [s for s in stack if "sehip" in s or "tools/" in s or "tests/" in s]
        where = " <- ".join(frames[:3]) if frames else (stack[0] if stack else "?")
        for f in fams:
            counts[(f, ev.name, where)] += 1
            total[f] += 1
    print(f"config {a.config}: {sum(total.values())} non-HIP kernel launches in one step")
    for (f, op, where), n in counts.most_common():
        print(f"{n:5d}  {f}\n       op={op}  at {where}")
    # the Python lines of the ATen ops that can launch a kernel (a dispatch mode sees the
    # backward's ops too: the autograd engine carries the mode to its threads)
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    meta = ("empty", "view", "_unsafe_view", "as_strided", "transpose", "t", "permute", "expand", "slice",
            "select", "unsqueeze", "squeeze", "detach", "alias", "reshape", "split", "chunk", "unbind",
            "lift_fresh", "empty_strided", "new_empty", "new_empty_strided", "set_", "is_same_size",
            "_local_scalar_dense", "record_stream", "empty_like", "_reshape_alias", "split_with_sizes",
            "unflatten", "flatten", "narrow", "diagonal", "view_as", "expand_as", "sym_size", "sym_stride",
            "sym_numel", "sym_storage_offset", "is_contiguous", "_has_compatible_shallow_copy_type")
    seen = collections.Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.__name__.split(".")[0]
            dev = [t for t in args if isinstance(t, torch.Tensor)]
            if name not in meta and any(t.is_cuda for t in dev):
                fr = [f"{os.path.basename(x.filename)}:{x.lineno}" for x in traceback.extract_stack()
                      if "sehip" in x.filename or "/tools/" in x.filename]
                seen[(func.__name__, " <- ".join(fr[-3:][::-1]))] += 1
            return func(*args, **(kwargs or {}))
    with ctx, Log():
        fn()
        torch.cuda.synchronize()
    print("ATen ops with a CUDA tensor argument (op, innermost sehip frames):")
    for (op, where), n in seen.most_common():
        print(f"{n:5d}  {op}  at {where}")


if __name__ == "__main__":
    main()
