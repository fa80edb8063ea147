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
(`f32_exact`) and the coarser split-bf16 / one-term bf16 steps
(`other_conv_math`) are timed beside it.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line. `value` = utterances processed by all ranks
during the K timed steps / max-over-ranks wall time. `roofline` is measured
live with HIP events around the complex-conv GEMM entry points during the
timed region; `cpu_baseline` times the oracle (the pure-PyTorch CPU port)
on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))

import torch  # noqa: E402

METRIC = "utterances/sec (4s@16kHz) FRCRN train at 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32-in MFMA dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: bf16 MFMA dense peak (no sparsity)
KERNEL_OF = {   # OpTimer tag -> (rocprof kernel name, description)
    "conv_fwd_f32": ("gather_gemm_kernel", "gather_gemm_kernel (se_conv2d_fwd, fp32 MFMA 32x32x2)"),
    "conv_data_f32": ("gather_gemm_kernel", "gather_gemm_kernel (se_conv2d_bwd_data, fp32 MFMA 32x32x2)"),
    "conv_fwd_bf16x3": ("gather_x3_kernel", "gather_x3_kernel (se_conv2d_fwd, split-bf16 MFMA 32x32x16 x3)"),
    "conv_fwd_bf16x6": ("gather_x6_kernel", "gather_x6_kernel (se_conv2d_fwd, 3-way split-bf16 MFMA 32x32x16 x6)"),
    "conv_data_bf16x6": ("gather_x6_kernel",
                         "gather_x6_kernel (se_conv2d_bwd_data, 3-way split-bf16 MFMA 32x32x16 x6)"),
    "conv_data_bf16x3": ("gather_x3_kernel",
                         "gather_x3_kernel (se_conv2d_bwd_data, split-bf16 MFMA 32x32x16 x3)"),
    "conv_wgrad_f32": ("wgrad_gemm_kernel", "wgrad_gemm_kernel (se_conv2d_bwd_weight, fp32 MFMA 32x32x2)"),
    "conv_wgrad_bf16x3": ("wgrad_x3_kernel",
                          "wgrad_x3_kernel (se_conv2d_bwd_weight, split-bf16 MFMA 32x32x16 x3)"),
    "conv_fwd_bf16": ("gather_x3_kernel", "gather_x3_kernel<TERMS=1> (se_conv2d_fwd, bf16 MFMA 32x32x16)"),
    "conv_data_bf16": ("gather_x3_kernel", "gather_x3_kernel<TERMS=1> (se_conv2d_bwd_data, bf16 MFMA 32x32x16)"),
    "conv_wgrad_bf16": ("wgrad_x3_kernel", "wgrad_x3_kernel<TERMS=1> (se_conv2d_bwd_weight, bf16 MFMA 32x32x16)"),
    "conv_fwd_f16x3": ("gather_x3_kernel", "gather_x3_kernel<F16> (se_conv2d_fwd, scaled split-fp16 MFMA 32x32x16 x3)"),
    "conv_data_f16x3": ("gather_x3_kernel",
                        "gather_x3_kernel<F16> (se_conv2d_bwd_data, scaled split-fp16 MFMA 32x32x16 x3)"),
    "conv_wgrad_f16x3": ("wgrad_x3_kernel",
                         "wgrad_x3_kernel<F16> (se_conv2d_bwd_weight, scaled split-fp16 MFMA 32x32x16 x3)"),
}
TERMS_OF = {"bf16x3": 3, "bf16x6": 6, "bf16": 1, "f16x3": 3}   # MFMA terms per fp32 product (peak divisor)
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E spec peak
SR, SECONDS = 16000, 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="utterances per GPU")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-op-timing", action="store_true")
    ap.add_argument("--compare", default="f32;bf16x3;bf16",
                    help="';'-separated conv math modes timed beside the default step (untimed by the "
                         "op timer): all-fp32 MFMA and the one-term bf16 GEMMs; '' for none")
    ap.add_argument("--no-compare", "--no-compare-f32", dest="compare", action="store_const", const="",
                    help="skip the comparison runs")
    ap.add_argument("--math", default=os.environ.get("SEHIP_CONV_MATH"),
                    help="conv GEMM MFMA form (se_conv2d_desc.math): f32, bf16x3, or per pass "
                         "'fwd=bf16x3,data=f32,weight=bf16x3'")
    return ap.parse_args()


def cpu_baseline(batch, steps):
    """Oracle (pure-PyTorch CPU restatement of the reference, pinned by the
    golden fixtures) timed on this box's host cores: a bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import models as O, train as OT
    from sehip.data import synthetic_pairs
    threads = torch.get_num_threads()
    noisy, clean = synthetic_pairs(batch, SR * SECONDS, seed=99, device="cpu")
    m = O.FRCRN().train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-2)
    OT.train_step(m, opt, noisy, clean)                     # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        OT.train_step(m, opt, noisy, clean)
    dt = time.perf_counter() - t0
    return {"value": batch * steps / dt, "unit": "utterances/sec", "cores": threads, "kind": "port",
            "sample": f"{steps} oracle FRCRN train steps (fwd+SI-SNR+bwd+clip+AdamW, fp32, "
                      f"B={batch} x 4 s @ 16 kHz) after 1 warm-up step, torch CPU, {threads} threads",
            "seconds": dt}


def main():
    args = parse()
    from sehip import functional as SF
    from sehip.data import synthetic_pairs
    from sehip.models import FRCRN
    from sehip.train import make_optimizer, setup_distributed, train_step, wrap_ddp

    if args.math:
        SF.set_conv_math(args.math)
    rank, world, local, device = setup_distributed()
    if device.type != "cuda":
        raise SystemExit("bench.py needs a GPU")
    torch.manual_seed(2023 + rank)
    model = FRCRN().to(device).train()
    model = wrap_ddp(model, device)
    opt = make_optimizer(model)
    B, L = args.batch, SR * SECONDS
    batches = [synthetic_pairs(B, L, seed=2023 + rank * 1_000_003 + i, device=device) for i in range(2)]

    for i in range(args.warmup):
        noisy, clean = batches[i % 2]
        train_step(model, opt, noisy, clean)
    torch.cuda.synchronize()

    timer = None if args.no_op_timing else SF.OpTimer()
    dist = torch.distributed if (world > 1 and torch.distributed.is_initialized()) else None
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    SF.set_op_timer(timer)
    t0 = time.perf_counter()
    for i in range(args.steps):
        noisy, clean = batches[i % 2]
        loss = train_step(model, opt, noisy, clean)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    SF.set_op_timer(None)
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_v = float(loss)
    kern = timer.summary() if timer else {}
    # ConvSTFT is a ~50 us kernel: per-call events inside the step also catch host
    # launch gaps, so its roofline uses 20 back-to-back launches between one
    # event pair, after the timed region (GPU-bound, comparable to rocprof's
    # per-kernel average)
    stft_burst_ms = None
    if timer and rank == 0:
        stft_mod = (model.module if hasattr(model, "module") else model).stft
        with torch.no_grad():
            x0 = batches[0][0]
            stft_mod(x0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                stft_mod(x0)
            e1.record()
            torch.cuda.synchronize()
            stft_burst_ms = e0.elapsed_time(e1) / 20

    # the same step with every conv pass in another MFMA form (untimed by the op
    # timer): "f32" = exact fp32 products everywhere; "bf16" = one-term bf16
    # operands (fp32 storage/accumulation), the speed form of SURVEY §8d config 4
    compare = {}
    default_mode = SF.get_conv_math()
    for mode in [m for m in args.compare.split(";") if m and m != default_mode]:
        SF.set_conv_math(mode)
        noisy, clean = batches[0]
        train_step(model, opt, noisy, clean)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(args.steps):
            noisy, clean = batches[i % 2]
            lc = train_step(model, opt, noisy, clean)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        e2 = time.perf_counter() - t1
        if dist:
            t = torch.tensor([e2], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e2 = float(t.item())
        compare[mode] = {"conv_math": mode, "value": round(world * B * args.steps / e2, 3),
                         "ms_per_step": round(1e3 * e2 / args.steps, 3), "final_loss": round(float(lc), 4)}
    SF.set_conv_math(default_mode)

    if rank != 0:
        return
    value = world * B * args.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "utterances/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": _dtype_label(SF.get_conv_math()),
        "data": "synthetic: on-device 4 s @ 16 kHz harmonic+AM clean / Gaussian-noise pairs at "
                "SNR U{-5..20} dB, random-init FRCRN (no datasets/checkpoints offline)",
        "config": {"workload": "FRCRN train step: fwd + SI-SNR + bwd + clip_grad_norm 0.5 + AdamW "
                               "(320/160/640 STFT, 4 s @ 16 kHz)",
                   "per_gpu_batch": B, "global_batch": B * world, "seq_len": L,
                   "parallelism": f"dp{world}"},
        "final_loss": round(loss_v, 4),
        "conv_math": SF.get_conv_math(),
        "conv_math_note": "fp32 storage and accumulation everywhere; 'f16x3' scales each operand by a "
                          "per-tensor power of two, splits it into hi+lo fp16 and sums hi*hi+hi*lo+lo*hi "
                          "on fp16 MFMA (4.0e-7 rel-L2 per conv vs fp64; the exact-fp32 MFMA path "
                          "6.4e-7): fp32-class, so the step's conv FLOP rate may exceed the 157.3 TF "
                          "fp32 MFMA peak; 'bf16x3' = hi+lo bf16 (4.5e-6, not fp32-class); 'bf16x6' = "
                          "three-way bf16 split, six terms (5.5e-7); tests/test_gpu_conv_x3.py",
    }
    if "f32" in compare:
        out["f32_exact"] = compare.pop("f32")
    if compare:
        out["other_conv_math"] = list(compare.values())
    if kern:
        # dominant GEMM kernel = the conv pass/kernel with the most time in the step
        # among those on the main stream: the deferred weight-grads run on a side
        # stream beside the data-grad / CBN chain, so their event spans include
        # time the CUs spent on the other stream (op_breakdown marks them)
        convs = {k: v for k, v in kern.items() if k.startswith("conv_") and v["flops"]
                 and not v["side_calls"]}
        tag = max(convs, key=lambda k: convs[k]["ms"])
        g = convs[tag]
        ach = g["flops"] / (g["ms"] * 1e-3) / 1e12
        terms = TERMS_OF.get(tag.rsplit("_", 1)[-1], 0)
        split = terms > 0
        peak = BF16_MFMA_PEAK_TFLOPS / terms if split else FP32_MFMA_PEAK_TFLOPS
        out["roofline"] = {
            "bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(ach / peak, 4),
            "traffic": _pmc_traffic(KERNEL_OF[tag][0]),
            "kernel": KERNEL_OF[tag][1], "timer_tag": tag,
            "launch_calls": g["calls"], "avg_ms_per_call": round(g["ms"] / g["calls"], 4),
            "algorithmic_flops_per_call": g["flops"] / g["calls"],
            "algorithmic_bytes_per_call": g["bytes"] / g["calls"],
            "flops_convention": "algorithmic fp32 conv FLOPs (torch FlopCounterMode formula)"
                                + (f"; peak = bf16 dense MFMA peak / {terms} MFMA terms per fp32 product"
                                   if split else "")}
        st = kern.get("stft_fwd")
        if st and stft_burst_ms:
            per_call = st["bytes"] / st["calls"]
            gbs = per_call / (stft_burst_ms * 1e-3) / 1e9
            out["stft_roofline"] = {
                "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": _pmc_traffic("stft_fwd_ip_kernel"),
                "kernel": "stft_fwd_ip_kernel (se_stft_fwd)",
                "avg_ms_per_call": round(stft_burst_ms, 4),
                "timing": "20 back-to-back launches between one HIP event pair, after the timed region",
                "algorithmic_bytes_per_call": per_call}
        out["op_breakdown"] = {
            k: {"calls": v["calls"], "ms_per_step": round(v["ms"] / args.steps, 3),
                **({"tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2)} if v["flops"] else {}),
                **({"gbs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1)} if v["bytes"] else {}),
                **({"side_stream_calls": v["side_calls"]} if v["side_calls"] else {})}
            for k, v in kern.items()}
        total_conv = sum(v["flops"] for k, v in kern.items() if k.startswith("conv"))
        out["conv_flops_per_utt"] = total_conv / (B * args.steps)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_batch, args.cpu_steps)
    print(json.dumps(out), flush=True)


FP32_CLASS = {"f32", "f16x3", "bf16x6"}   # per-conv error at or below the exact-fp32 MFMA path's


def _dtype_label(mode):
    """The arithmetic the step computes in: "f32" only for exact fp32 products;
    fp32-class emulations name their split form; anything coarser is labelled
    by its narrowest pass."""
    modes = {kv.split("=")[1] for kv in mode.split(",") if "=" in kv and not kv.startswith("fwd_dec_min")} \
        if "=" in mode else {mode}
    if modes == {"f32"}:
        return "f32"
    if modes <= FP32_CLASS:
        return "f32-class (" + "+".join(sorted(modes - {"f32"})) + " split MFMA, fp32 storage/accumulate)"
    return "mixed (" + "+".join(sorted(modes)) + "; not fp32-class)"


def _pmc_traffic(kernel):
    """HBM bytes per launch from the committed PMC summary (tools/pmc_summary.py
    -> profiles/pmc_traffic.json), or None when not collected."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
