#!/usr/bin/env python3
"""FRCRN training throughput on MI355X — BASELINE.json's metric.

One step = one FRCRN training iteration (trainer.py:99-124 + 210-221:
forward, SI-SNR, backward, clip_grad_norm_(0.5), AdamW) on 64 synthetic
4 s @ 16 kHz noisy/clean pairs per GPU, inputs resident in HBM.
fp32 storage and accumulation throughout (the reference's precision; parity
is judged at 1e-4 fp32). The conv GEMMs' MFMA form follows SEHIP_CONV_MATH /
--math; the default "f16x3" (scaled split-fp16, three MFMA terms) is
fp32-class on every pass: each pass's error against fp64 is 0.63-0.70x the
exact-fp32 MFMA path's (tests/test_gpu_conv_x3.py). The all-fp32-MFMA step
(`f32_exact`, with its own warm-up and roofline) and the coarser split-bf16 /
one-term bf16 steps (`other_conv_math`) are timed beside it.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line. `value` = utterances processed by all ranks
during the K timed steps / max-over-ranks wall time, measured with no
instrumentation inside the timed region. A second pass of K steps with HIP
events around every C-ABI call (on the launching stream) gives the per-op
breakdown and the live `roofline` of the dominant GEMM kernel; its PMC HBM
traffic comes from the committed rocprofv3 summary of the same kernel
instantiation (profiles/pmc_traffic.json). `cpu_baseline` times the oracle
(the pure-PyTorch CPU port) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))

import torch  # noqa: E402

METRIC = "utterances/sec (4s@16kHz) FRCRN train at 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32-in MFMA dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: bf16 / f16 MFMA dense peak (no sparsity)
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E spec peak
SR, SECONDS = 16000, 4
PROFILE_STATS = os.path.join(ROOT, "profiles", "r6_bench_kernel_stats.csv")
# the ConvSTFT / iSTFT kernels of the STFT rooflines (se_stft_fwd: the register-radix form
# for nfft 640)
STFT_KERNELS = (("stft_fwd", "stft_fwd_rg_kernel"), ("istft_fwd", "istft_fwd_wv_kernel"),
                ("istft_bwd", "istft_bwd_rg_kernel"))

# OpTimer tag -> (kernel instantiation as rocprof names it, launches per call, description).
# The decoder's joined passes are one launch of one instantiation per call (the data-grad of
# a stride-(2,1) convT is a single strided class; its 256 columns take the 8-wave NW = 2
# tile), so their event time and their PMC bytes describe the same launches. Other tags
# share their instantiation with other passes: no traffic is attributed to them.
KERNEL_OF = {
    "conv_data_joined_f16x3": ("gather_x3_kernel<true, 3, 2, 2, true, 0>", 1,
                               "gather_x3_kernel<F16, joined data-grad> (se_conv2d_bwd_data_joined, "
                               "scaled split-fp16 MFMA 32x32x16 x3)"),
    "conv_fwd_joined_f16x3": ("gather_x3_kernel<true, 3, 1, 1, true, 0>", 2,
                              "gather_x3_kernel<F16, joined fwd> (se_conv2d_fwd_joined, 2 stride-phase "
                              "launches per call)"),
    "conv_wgrad_joined_f16x3": ("wgrad_x3_kernel<true, 3, true, true, 2, false, 0, 2>", 1,
                                "wgrad_x3_kernel<F16, joined, 256 x 256 tiles> (se_conv2d_bwd_weight_joined)"),
    "conv_data_joined_bf16x3": ("gather_x3_kernel<true, 3, 2, 2, false, 0>", 1,
                                "gather_x3_kernel<bf16x3, joined data-grad> (se_conv2d_bwd_data_joined)"),
    "conv_data_joined_f32": (None, 1, "gather_gemm_kernel<128, 128, 2, 2, true> on the materialised join "
                                      "(se_conv2d_bwd_data + se_complex_join_bwd, fp32 MFMA 32x32x2)"),
    "conv_data_f32": (None, 1, "gather_gemm_kernel (se_conv2d_bwd_data, fp32 MFMA 32x32x2)"),
    "conv_fwd_f32": (None, 1, "gather_gemm_kernel (se_conv2d_fwd, fp32 MFMA 32x32x2)"),
    "conv_fwd_joined_f32": (None, 2, "gather_gemm_kernel on the materialised join (se_conv2d_fwd)"),
    "conv_data_f16x3": (None, 1, "gather_x3_kernel<F16> (se_conv2d_bwd_data, encoder layers)"),
    "conv_fwd_f16x3": (None, 1, "gather_x3_kernel<F16> (se_conv2d_fwd, encoder layers)"),
}
TERMS_OF = {"bf16x3": 3, "bf16x6": 6, "bf16": 1, "f16x3": 3}   # MFMA terms per fp32 product
FP32_CLASS = {"f32", "f16x3", "bf16x6"}   # per-conv error at or below the exact-fp32 MFMA path's


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="utterances per GPU")
    ap.add_argument("--cpu-steps", type=int, default=20, help="timed oracle steps (BASELINE.md plan: >= 20)")
    ap.add_argument("--cpu-warmup", type=int, default=5, help="untimed oracle steps first (BASELINE.md plan: 5)")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-budget-s", type=float, default=400.0,
                    help="wall-clock cap of the CPU baseline (warm-up + timed); the timed loop stops early "
                         "past it and the sample says how many steps ran")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-op-timing", action="store_true")
    ap.add_argument("--compare", default="f32;bf16",
                    help="';'-separated conv math modes timed beside the default step: the all-fp32 MFMA "
                         "step (reported as f32_exact, with its own warm-up and roofline) and the coarser "
                         "split-bf16 / one-term bf16 steps (bf16 = SURVEY 8(d) config 4's 'bf16 (speed)' "
                         "leg, reported as bf16_speed); '' for none")
    ap.add_argument("--no-compare", "--no-compare-f32", dest="compare", action="store_const", const="",
                    help="skip the comparison runs")
    ap.add_argument("--math", default=os.environ.get("SEHIP_CONV_MATH"),
                    help="conv GEMM MFMA form (se_conv2d_desc.math): f16x3, f32, bf16x3, or per pass "
                         "'fwd=f16x3,data=f32,weight=f16x3'")
    return ap.parse_args()


def _dtype_label(mode):
    """The arithmetic the step computes in: "f32" only for exact fp32 products;
    fp32-class emulations name their split form; anything coarser is labelled
    by its passes."""
    modes = {kv.split("=")[1] for kv in mode.split(",") if "=" in kv and not kv.startswith("fwd_dec_min")} \
        if "=" in mode else {mode}
    if modes == {"f32"}:
        return "f32"
    if modes <= FP32_CLASS:
        return "f32-class (" + "+".join(sorted(modes - {"f32"})) + " split MFMA, fp32 storage/accumulate)"
    return "mixed (" + "+".join(sorted(modes)) + "; not fp32-class)"


def _note(msg):
    """Progress on stderr (the JSON line stays alone on stdout): a long phase such as the
    CPU baseline must not look like a hung command to a watchdog."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cpu_threads():
    """BASELINE.md's plan: len(os.sched_getaffinity(0)) threads, capped by
    OMP_NUM_THREADS where the job sets it (the GPU box's CPU share is 16 cores
    while the affinity mask lists the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff), aff


def cpu_baseline(batch, steps, warmup, budget_s):
    """Oracle (pure-PyTorch CPU restatement of the reference, pinned by the
    golden fixtures) timed on this box's host cores: BASELINE.md's CPU-baseline
    plan (B = 8 FRCRN train steps, 5 warm-up + 20 timed, fp32), under a wall-clock
    cap so the default bench stays bounded."""
    sys.path.insert(0, ROOT)
    from oracle import models as O, train as OT
    from sehip.data import synthetic_pairs
    threads, affinity = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        noisy, clean = synthetic_pairs(batch, SR * SECONDS, seed=99, device="cpu")
        m = O.FRCRN().train()
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-2)
        t_start = time.perf_counter()
        for i in range(warmup):
            OT.train_step(m, opt, noisy, clean)
            _note(f"cpu baseline warm-up step {i + 1}/{warmup}")
        t_warm = time.perf_counter() - t_start
        per_step = t_warm / max(warmup, 1)
        t0 = time.perf_counter()
        done = 0
        for _ in range(steps):
            if done and time.perf_counter() - t_start + per_step > budget_s:
                break
            OT.train_step(m, opt, noisy, clean)
            done += 1
            _note(f"cpu baseline step {done}/{steps}")
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return {"value": round(batch * done / dt, 4), "unit": "utterances/sec", "cores": threads, "kind": "port",
            "sample": f"{done} timed oracle FRCRN train steps (fwd+SI-SNR+bwd+clip+AdamW, fp32, B={batch} x 4 s "
                      f"@ 16 kHz) after {warmup} warm-up steps, torch CPU, {threads} threads"
                      + (f" (stopped at the {budget_s:.0f} s cap; {steps} planned)" if done < steps else ""),
            "cpu_model": _cpu_model(), "affinity_cpus": affinity, "seconds": round(dt, 2),
            "warmup_seconds": round(t_warm, 2)}


_ROCTX: list = []


def _roctx():
    """librocprofiler-sdk-roctx when SEHIP_ROCTX_REGIONS=1: the uninstrumented timed steps run
    inside a roctx range "timed", which `rocprofv3 --marker-trace` records beside the kernel
    trace; tools/region_stats.py keeps the kernels inside it (no data generation, model
    construction or warm-up in the kernel statistics)."""
    if os.environ.get("SEHIP_ROCTX_REGIONS") != "1":
        return None
    if not _ROCTX:
        import ctypes
        lib = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
        lib.roctxRangePushA.argtypes, lib.roctxRangePushA.restype = [ctypes.c_char_p], ctypes.c_int
        lib.roctxRangePop.argtypes, lib.roctxRangePop.restype = [], ctypes.c_int
        _ROCTX.append(lib)
    return _ROCTX[0]


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:   # noqa: BLE001 (reported, not needed)
        return None


def _kernel_key(name):
    """rocprof kernel name -> 'base<template args>' (the key of profiles/pmc_traffic.json)."""
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    depth, end = 0, len(name)
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            end = i
            break
    return name[:end].split("::")[-1].strip() if "<" not in name[:end] else name[:end].strip()


def _rocprof_avg_ms(kernel):
    """Average duration of one kernel (exact instantiation, or every instantiation of a
    base name) in the committed rocprofv3 --stats summary, or None."""
    try:
        with open(PROFILE_STATS) as f:
            rows = [r for r in csv.DictReader(f)
                    if _kernel_key(r["Name"]) == kernel or _kernel_key(r["Name"]).split("<")[0] == kernel]
    except (OSError, KeyError):
        return None
    calls = sum(int(r["Calls"]) for r in rows)
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    return round(total / calls / 1e6, 4) if calls else None


def _pmc(kernel):
    """PMC HBM bytes per launch of one kernel instantiation (or base name) from the
    committed summary (tools/pmc_summary.py -> profiles/pmc_traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel)
    except (OSError, ValueError):
        return None


def _roofline(kern, steps, side_ok=False):
    """Live roofline of the conv pass (OpTimer tag) with the most event time among the
    main-stream ones (the deferred weight-grads run on a side stream beside the
    data-grad / CBN chain, so their event spans include time the CUs spent on the other
    stream; side_ok=True looks at those)."""
    convs = {k: v for k, v in kern.items() if k.startswith("conv_") and v["flops"]
             and (side_ok or not v["side_calls"])}
    if not convs:
        return None
    tag = max(convs, key=lambda k: convs[k]["ms"])
    g = convs[tag]
    ach = g["flops"] / (g["ms"] * 1e-3) / 1e12
    terms = TERMS_OF.get(tag.rsplit("_", 1)[-1], 0)
    # split forms: the kernel issues `terms` fp16 / bf16 MFMA products per fp32 product, so
    # its MFMA rate is terms x the fp32-equivalent rate, against the dense fp16 / bf16 peak
    ach32 = ach
    ach = ach32 * terms if terms else ach32
    peak = BF16_MFMA_PEAK_TFLOPS if terms else FP32_MFMA_PEAK_TFLOPS
    kname, per_call, desc = KERNEL_OF.get(tag, (None, 1, tag))
    launches = g["calls"] * per_call
    alg_bytes_launch = g["bytes"] / launches
    pmc = _pmc(kname) if kname else None
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    out = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
           "frac": round(ach / peak, 4), "traffic": traffic,
           "achieved_fp32_equivalent": round(ach32, 2),
           "kernel": desc, "kernel_instantiation": kname, "timer_tag": tag,
           "calls_per_step": g["calls"] / steps, "launches_per_step": launches / steps,
           "avg_ms_per_launch": round(g["ms"] / launches, 4),
           "algorithmic_flops_per_launch": g["flops"] / launches,
           "algorithmic_bytes_per_launch": alg_bytes_launch,
           "traffic_per_step": traffic * launches / steps if traffic else None,
           "algorithmic_bytes_per_step": g["bytes"] / steps,
           "traffic_over_algorithmic": round(traffic / alg_bytes_launch, 3) if traffic else None,
           "rocprof_avg_ms_per_launch": _rocprof_avg_ms(kname) if kname else None,
           "flops_convention": "algorithmic fp32 conv FLOPs (torch FlopCounterMode formula)"
                               + (f" x {terms} MFMA terms per fp32 product = fp16/bf16 MFMA FLOPs issued; "
                                  "peak = dense fp16/bf16 MFMA peak (achieved_fp32_equivalent = the fp32 "
                                  "conv rate)" if terms else "; peak = fp32 MFMA dense peak"),
           "bytes_convention": "algorithmic bytes = one read of each input, one write of each output "
                               "(fp32); traffic = PMC FETCH_SIZE x2 (gfx950) + WRITE_SIZE per launch of "
                               "that instantiation; avg_ms_per_launch = HIP-event span per call / "
                               "launches per call (includes the call's small prologue kernels)"}
    if kname is None:
        out["traffic_note"] = "instantiation shared with other passes: no PMC bytes attributed"
    return out


def _breakdown(kern, steps):
    return {k: {"calls": v["calls"], "ms_per_step": round(v["ms"] / steps, 3),
                **({"tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2)} if v["flops"] else {}),
                **({"gbs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1)} if v["bytes"] else {}),
                **({"side_stream_calls": v["side_calls"]} if v["side_calls"] else {})}
            for k, v in kern.items()}


def main():
    """`--gpus N` is the world size. Under torchrun (WORLD_SIZE set) it must equal
    WORLD_SIZE. Without torchrun and N > 1, this process spawns the N ranks itself
    (sehip.train.spawn_ranks: one fresh process per GPU, RCCL) after checking,
    without initialising the GPU, that N GPUs are visible; it never silently runs
    fewer ranks than asked."""
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        visible = torch.cuda.device_count()      # counts devices without initialising them
        if visible < args.gpus:
            raise SystemExit(f"bench.py --gpus {args.gpus}: only {visible} GPU(s) visible; refusing to run "
                             f"fewer ranks than asked")
        from sehip.train import spawn_ranks
        spawn_ranks(args.gpus, run, (args,))
        return
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={env_world}")
    run(args)


def run(args):
    from sehip import functional as SF
    from sehip.data import synthetic_pairs
    from sehip.models import FRCRN
    from sehip.train import make_optimizer, setup_distributed, train_step, wrap_ddp

    if args.math:
        SF.set_conv_math(args.math)
    rank, world, local, device = setup_distributed()
    if device.type != "cuda":
        raise SystemExit("bench.py needs a GPU")
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} rank(s)")
    dist_backend = torch.distributed.get_backend() if world > 1 else None
    torch.manual_seed(2023 + rank)
    model = FRCRN().to(device).train()
    model = wrap_ddp(model, device)
    opt = make_optimizer(model)
    B, L = args.batch, SR * SECONDS
    batches = [synthetic_pairs(B, L, seed=2023 + rank * 1_000_003 + i, device=device) for i in range(2)]
    dist = torch.distributed if (world > 1 and torch.distributed.is_initialized()) else None

    trace = os.environ.get("SEHIP_BENCH_TRACE") == "1"

    def timed(steps, warmup, timer=None):
        for i in range(warmup):
            noisy, clean = batches[i % 2]
            train_step(model, opt, noisy, clean)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        SF.set_op_timer(timer)
        rt = _roctx() if timer is None else None
        if rt is not None:
            rt.roctxRangePushA(b"timed")
        t0 = time.perf_counter()
        marks = []
        for i in range(steps):
            noisy, clean = batches[i % 2]
            loss = train_step(model, opt, noisy, clean)
            if trace:
                marks.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        if rt is not None:
            rt.roctxRangePop()
        if trace:   # host enqueue timeline (SEHIP_BENCH_TRACE=1): where the host blocked
            _note("enqueue ms: " + " ".join(f"{1e3 * m:.0f}" for m in marks)
                  + f" | sync {1e3 * (time.perf_counter() - t0):.0f}")
            ms = torch.cuda.memory_stats(device)
            _note(f"allocator: reserved peak {ms['reserved_bytes.all.peak'] / 2**30:.1f} GiB, allocated peak "
                  f"{ms['allocated_bytes.all.peak'] / 2**30:.1f} GiB, alloc retries {ms['num_alloc_retries']}, "
                  f"device mallocs {ms['segment.all.allocated']}")
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        SF.set_op_timer(None)
        if dist:
            t = torch.tensor([elapsed], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, float(loss)

    default_mode = SF.get_conv_math()
    _note(f"rank {rank}: {args.warmup} warm-up + {args.steps} timed steps")
    elapsed, loss_v = timed(args.steps, args.warmup)            # the headline: no instrumentation
    _note(f"rank {rank}: {world * B * args.steps / elapsed:.1f} utt/s")
    kern, kern_iso = {}, {}
    if not args.no_op_timing:
        timer = SF.OpTimer()
        timed(args.steps, 0, timer)
        kern = timer.summary()
        # the same kernels with the side streams off (SEHIP_OVERLAP=0): each GEMM's own rate,
        # without the deferred weight-grads / CCBAM gates taking CU slots beside it
        prev = os.environ.get("SEHIP_OVERLAP")
        os.environ["SEHIP_OVERLAP"] = "0"
        timer = SF.OpTimer()
        timed(args.steps, 1, timer)
        kern_iso = timer.summary()
        _note(f"rank {rank}: op timing done")
        if prev is None:
            del os.environ["SEHIP_OVERLAP"]
        else:
            os.environ["SEHIP_OVERLAP"] = prev

    # ConvSTFT / iSTFT are ~30-50 us kernels: per-call events inside the step also catch host
    # launch gaps, so each kernel is timed here on its own, live in this run: a burst of 50
    # back-to-back launches between two HIP events on the launching stream (the per-launch
    # average: the event edges amortised, the launches queued ahead of the GPU), plus the median
    # of 20 single-launch spans (one event pair around ONE launch on an idle device). The
    # roofline frac uses the burst average; the committed rocprofv3 --stats average of the same
    # kernel is reported beside it as a reference only.
    bursts = {}
    if kern and rank == 0:
        mod = model.module if hasattr(model, "module") else model
        x0 = batches[0][0]

        def burst(fn, n=50):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n, sorted(ts)[len(ts) // 2]

        # the kernels launched straight into preallocated buffers (the launch helpers the
        # autograd Functions call): per-call host work (autograd, allocation) would
        # otherwise set the pace of a 30-60 us kernel
        st_m, is_m = mod.stft, mod.istft
        x2 = (x0[:, 0] if x0.dim() == 3 else x0).contiguous()
        with torch.no_grad():
            spec = st_m(x0)
            wav = is_m(spec)
        off = is_m.pad if is_m.center else 0
        wav_buf, gspec = torch.empty_like(wav), torch.empty_like(spec)
        gw = torch.randn(wav.shape, device=device)
        bursts["stft_fwd"] = burst(lambda: SF.stft_launch(x2, spec, None, st_m._win, st_m._tw, st_m.window_size,
                                                          st_m.hop_size, st_m.fft_size, st_m.center, False))
        bursts["istft_fwd"] = burst(lambda: SF.istft_launch(spec, wav_buf, is_m._win, is_m._tw, is_m.window_size,
                                                            is_m.hop_size, is_m.fft_size, off, wav.shape[-1]))
        bursts["istft_bwd"] = burst(lambda: SF.istft_bwd_launch(gw, gspec, is_m._win, is_m._tw, is_m.window_size,
                                                                is_m.hop_size, is_m.fft_size, off, wav.shape[-1]))

    # the same step in other MFMA forms: "f32" = exact fp32 products everywhere (own warm-up
    # and roofline); "bf16x3" / "bf16" = the coarser split-bf16 / one-term bf16 GEMMs
    compare = {}
    for mode in [m for m in args.compare.split(";") if m and m != default_mode]:
        SF.set_conv_math(mode)
        wu = max(args.warmup, 1) if mode == "f32" else 1
        e2, lc = timed(args.steps, wu)
        _note(f"rank {rank}: {mode} leg {world * B * args.steps / e2:.1f} utt/s")
        entry = {"conv_math": mode, "dtype": _dtype_label(mode), "value": round(world * B * args.steps / e2, 3),
                 "ms_per_step": round(1e3 * e2 / args.steps, 3), "warmup": wu, "final_loss": round(lc, 4)}
        if mode == "f32" and not args.no_op_timing:
            timer = SF.OpTimer()
            timed(args.steps, 0, timer)
            entry["roofline"] = _roofline(timer.summary(), args.steps)
        compare[mode] = entry
    SF.set_conv_math(default_mode)

    if rank != 0:
        return
    value = world * B * args.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "utterances/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": _dtype_label(default_mode),
        "data": "synthetic: on-device 4 s @ 16 kHz harmonic+AM clean / Gaussian-noise pairs at "
                "SNR U{-5..20} dB, random-init FRCRN (no datasets/checkpoints offline)",
        "config": {"workload": "FRCRN train step: fwd + SI-SNR + bwd + clip_grad_norm 0.5 + AdamW "
                               "(320/160/640 STFT, 4 s @ 16 kHz)",
                   "per_gpu_batch": B, "global_batch": B * world, "seq_len": L,
                   "parallelism": f"dp{world}"},
        "final_loss": round(loss_v, 4),
        "dist": ({"world": world, "backend": dist_backend, "rccl_version": _rccl_version(),
                  "launcher": ("torchrun" if os.environ.get("TORCHELASTIC_RUN_ID")
                               else "bench.py spawn" if os.environ.get("SEHIP_SPAWNED") else "env")}
                 if world > 1 else None),
        "conv_math": default_mode,
        "conv_math_note": "fp32 storage and accumulation everywhere; 'f16x3' scales each operand by a "
                          "per-tensor power of two, splits it into hi+lo fp16 and sums hi*hi+hi*lo+lo*hi "
                          "on fp16 MFMA (4.0e-7 rel-L2 per conv vs fp64; the exact-fp32 MFMA path "
                          "6.4e-7): fp32-class, so the step's conv FLOP rate may exceed the 157.3 TF "
                          "fp32 MFMA peak; 'bf16x3' = hi+lo bf16 (4.5e-6, not fp32-class); 'bf16x6' = "
                          "three-way bf16 split, six terms (5.5e-7); tests/test_gpu_conv_x3.py",
        "timing_note": "value: K steps with no instrumentation; roofline / op_breakdown: a second pass "
                       "of K steps with HIP events around every C-ABI call; roofline_isolated: a third "
                       "pass with the side streams off",
    }
    if "f32" in compare:
        out["f32_exact"] = compare.pop("f32")
    if "bf16" in compare:   # "fp32 (parity) and bf16 (speed)"
        out["bf16_speed"] = compare.pop("bf16")
        out["bf16_speed"]["note"] = ("the same FRCRN train step with every conv GEMM on one-term bf16 MFMA "
                                     "(operands rounded to bf16, fp32 accumulate and storage: the arithmetic "
                                     "of a bf16 autocast conv); not fp32-class, not the headline")
    if compare:
        out["other_conv_math"] = list(compare.values())
    if kern:
        out["roofline"] = _roofline(kern, args.steps)
        out["roofline_side_stream"] = _roofline({k: v for k, v in kern.items() if "wgrad" in k},
                                                args.steps, side_ok=True)
        if kern_iso:
            tag = out["roofline"]["timer_tag"] if out["roofline"] else None
            iso = _roofline({tag: kern_iso[tag]} if tag in kern_iso else kern_iso, args.steps)
            if iso:
                iso["note"] = ("the same kernel in a third pass of K steps with the side streams off "
                               "(SEHIP_OVERLAP=0): its own rate; `roofline` above is its rate inside the "
                               "overlapped step, where the deferred weight-grads share the CUs")
            out["roofline_isolated"] = iso
            wg = {k: v for k, v in kern_iso.items() if "wgrad" in k}
            if wg:
                out["roofline_side_stream_isolated"] = _roofline(wg, args.steps, side_ok=True)
        for name, kname in STFT_KERNELS:
            st = kern.get(name)
            if not (st and name in bursts):
                continue
            per_call = st["bytes"] / st["calls"]
            rp = _rocprof_avg_ms(kname)
            dur, single = bursts[name]
            gbs = per_call / (dur * 1e-3) / 1e9
            pmc = _pmc(kname)
            out[f"{name}_roofline"] = {
                "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "kernel": f"{kname} (se_{name})", "duration_ms": round(dur, 4),
                "duration_source": "live, this run: HIP events around 50 back-to-back launches on the launching "
                                   "stream, divided by 50 (sehip.functional.*_launch into preallocated buffers, "
                                   "after the timed region)",
                "single_launch_event_ms": round(single, 4),
                "single_launch_note": "one HIP event pair around one launch on an idle device, median of 20 "
                                      "(includes the event / launch edges)",
                "reference_rocprof_avg_ms": rp,
                "reference_rocprof_source": (f"committed rocprofv3 --stats summary "
                                             f"({os.path.relpath(PROFILE_STATS, ROOT)}), a reference only: it "
                                             "may predate this build or come from another box") if rp else None,
                "algorithmic_bytes_per_call": per_call}
        out["op_breakdown"] = _breakdown(kern, args.steps)
        total_conv = sum(v["flops"] for k, v in kern.items() if k.startswith("conv"))
        out["conv_flops_per_utt"] = total_conv / (B * args.steps)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_batch, args.cpu_steps, args.cpu_warmup, args.cpu_budget_s)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
