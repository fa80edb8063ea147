"""BASELINE.json configs 2, 3 and 5 on one MI355X, one JSON line each (bench.py
is config 4, the headline). Synthetic inputs, random-init weights.

  2: DCUNet-16 inference, 4 s @ 16 kHz, batch 16, bf16 GEMM operands (SE_MATH_BF16)
  3: DCCRN-CL training step, 4 s @ 16 kHz, batch 64, bf16 GEMM operands
  5: CARN fp16 storage (model.half()) inference on 30 s @ 48 kHz = [1, 1,440,000],
     in 4 s chunks overlapping 50 ms (sehip/longform.py), and the same in fp32 and
     as one unchunked sequence (T = 9002 frames)

Configs 2 and 3 run twice: fp32 storage with bf16 GEMM operands, and as the
reference's bf16 run, model.to(torch.bfloat16) with bf16 activations end to end
(the CBN / STFT / BN kernels read and write bf16). Each line carries a roofline:
algorithmic conv FLOPs per utterance (DCUNet-16 36.8 GFLOP forward,
DCCRN-CL 199 GFLOP forward + backward) x utterances/s against the 2.5 PFLOP/s dense
bf16 MFMA peak.

Usage: python tools/bench_configs.py [--configs 2,3,5] [--iters 5] [--storage fp32,bf16]"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import torch


_ROCTX = []


def _roctx():
    """librocprofiler-sdk-roctx when SEHIP_ROCTX_REGIONS=1: the timed iterations run inside a
    roctx range "timed", which `rocprofv3 --marker-trace` records beside the kernel trace;
    tools/region_stats.py keeps the kernels inside it (no data generation, model construction
    or warm-up in the kernel statistics)."""
    if not _ROCTX:
        lib = None
        if os.environ.get("SEHIP_ROCTX_REGIONS") == "1":
            import ctypes
            lib = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
            lib.roctxRangePushA.argtypes, lib.roctxRangePushA.restype = [ctypes.c_char_p], ctypes.c_int
            lib.roctxRangePop.argtypes, lib.roctxRangePop.restype = [], ctypes.c_int
        _ROCTX.append(lib)
    return _ROCTX[0]


def timeit(fn, iters, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    rt = _roctx()
    if rt is not None:
        rt.roctxRangePushA(b"timed")
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    if rt is not None:
        rt.roctxRangePop()
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,5")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--storage", default="fp32,bf16")
    a = ap.parse_args()
    storages = a.storage.split(",")
    BF16_PEAK = 2500.0
    FLOPS = {2: 36.8e9, 3: 199e9}   # per utterance (torch FlopCounterMode)

    def roof(cfg, ups):
        tf = ups * FLOPS[cfg] / 1e12
        return {"bound": "mfma", "achieved": round(tf, 1), "peak": BF16_PEAK, "unit": "TFLOP/s",
                "frac": round(tf / BF16_PEAK, 4), "flops_per_utt": FLOPS[cfg]}
    from sehip import functional as F, models as M, longform as L
    from sehip.data import synthetic_pairs
    from sehip.train import make_optimizer, train_step
    dev = torch.device("cuda")
    cfgs = a.configs.split(",")
    for storage in storages:
        sdt = torch.bfloat16 if storage == "bf16" else torch.float32
        if "2" in cfgs:
            F.set_conv_math("bf16")
            m = M.DCUNet("dcunet16", 512, 128, 512).to(dev).eval().to(sdt)
            x, _ = synthetic_pairs(16, 64000, seed=5, device=dev)
            x = x.to(sdt)
            with torch.no_grad():
                dt = timeit(lambda: m(x), a.iters)
            print(json.dumps({"config": 2, "workload": "DCUNet-16 inference 4 s @ 16 kHz, batch 16",
                              "conv_math": "bf16", "storage": storage, "value": round(16 / dt, 2),
                              "unit": "utterances/sec", "ms_per_batch": round(dt * 1e3, 3),
                              "roofline": roof(2, 16 / dt)}), flush=True)
        if "3" in cfgs:
            F.set_conv_math("bf16")
            m = M.DCCRN("dccrn-CL", 400, 100, 512).to(dev).train().to(sdt)
            opt = make_optimizer(m)
            x, c = synthetic_pairs(64, 64000, seed=6, device=dev)
            x, c = x.to(sdt), c.to(sdt)
            dt = timeit(lambda: train_step(m, opt, x, c), a.iters)
            print(json.dumps({"config": 3, "workload": "DCCRN-CL train step 4 s @ 16 kHz, batch 64",
                              "conv_math": "bf16", "storage": storage, "value": round(64 / dt, 2),
                              "unit": "utterances/sec", "ms_per_step": round(dt * 1e3, 3),
                              "roofline": roof(3, 64 / dt)}), flush=True)
    def counted_flops(fn):
        """FLOPs of one call as the op timer records them (conv passes: torch
        FlopCounterMode's formula; LSTM: 2 L B T G H per recurrence), no timing."""
        timer = F.OpTimer()
        F.set_op_timer(timer)
        try:
            with torch.no_grad():
                fn()
            torch.cuda.synchronize()
        finally:
            F.set_op_timer(None)
        return sum(v.get("flops", 0.0) for v in timer.summary().values())

    def roof_of(flops, dt, peak, note):
        tf = flops / dt / 1e12
        return {"bound": "mfma", "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(tf / peak, 5), "flops_per_utt": flops, "note": note}

    if "5" in cfgs:
        F.set_conv_math(F.DEFAULT_CONV_MATH)
        sr, secs = 48000, 30
        x, _ = synthetic_pairs(1, sr * secs, sr=sr, seed=7, device=dev)
        chunk, overlap = 4 * sr, sr // 20
        for dtype, label in ((torch.float16, "fp16"), (torch.float32, "fp32")):
            m = M.CARN(320, 160, 512).to(dev).eval().to(dtype)
            xd = x.to(dtype)
            dt = timeit(lambda: L.enhance_chunked(m, xd, chunk, overlap), a.iters, warm=1)
            fl = counted_flops(lambda: L.enhance_chunked(m, xd, chunk, overlap))
            print(json.dumps({"config": 5, "workload": "CARN inference, 30 s @ 48 kHz [1, 1440000], 4 s chunks "
                              "(50 ms cross-fade) as one batch of 8", "storage": label,
                              "conv_math": F.get_conv_math(), "ms_per_utterance": round(dt * 1e3, 2),
                              "realtime_factor": round(secs / dt, 1), "value": round(1 / dt, 3),
                              "unit": "utterances/sec (30 s each)",
                              "roofline": roof_of(fl, dt, BF16_PEAK, "fp16 storage: one-term fp16 MFMA; fp32: "
                                                  "f16x3 (3 MFMA terms per FLOP counted once); the 512-wide "
                                                  "LSTM recurrence is latency-bound")}), flush=True)
        m = M.CARN(320, 160, 512).to(dev).eval().half()
        xh = x.half()   # the input in the model's storage type before the timed calls
        with torch.no_grad():
            dt = timeit(lambda: m(xh), max(1, a.iters // 2), warm=1)
        fl = counted_flops(lambda: m(xh))
        print(json.dumps({"config": 5, "workload": "CARN inference, 30 s @ 48 kHz as ONE sequence (T = 9002 frames)",
                          "storage": "fp16", "ms_per_utterance": round(dt * 1e3, 2),
                          "realtime_factor": round(secs / dt, 1),
                          "roofline": roof_of(fl, dt, BF16_PEAK, "dominated by the 9002-step LSTM recurrence "
                                              "(latency-bound: 2 us per step)")}), flush=True)


if __name__ == "__main__":
    main()
