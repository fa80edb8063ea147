"""Where one training step's time goes along its critical path, from a
rocprofv3 kernel trace: per stream, when it goes idle for the last time before
the optimizer, the kernels it runs in the step's last N ms, and the main
stream's phases (forward up to the loss, backward, optimizer).
   python tools/trace_tail.py <run_kernel_trace.csv> [tail ms, default 20]"""
import collections
import csv
import sys

from trace_step import key


def main(path, tail_ms=20.0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
    a, b = idx[-2] + 1, idx[-1] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    rel = lambda t: (int(t) - t0) / 1e6
    end = rel(step[-1]["End_Timestamp"])
    print(f"step span {end:.2f} ms")
    opt = [r for r in step if any(s in r["Kernel_Name"].lower() for s in ("adamw", "clip", "sumsq"))]
    if opt:
        print(f"optimizer kernels start at {rel(opt[0]['Start_Timestamp']):.2f} ms")
    sis = [r for r in step if "sisnr" in r["Kernel_Name"].lower()]
    if sis:
        print(f"SI-SNR kernels at {rel(sis[0]['Start_Timestamp']):.2f} ms (forward ends)")
    by = collections.defaultdict(list)
    for r in step:
        by[r["Stream_Id"]].append(r)
    for s, rs in sorted(by.items()):
        last = max(rel(r["End_Timestamp"]) for r in rs if r not in opt) if any(r not in opt for r in rs) else 0
        print(f"\n== stream {s}: last non-optimizer kernel ends at {last:.2f} ms")
        agg = collections.defaultdict(float)
        for r in rs:
            st, en = rel(r["Start_Timestamp"]), rel(r["End_Timestamp"])
            ov = min(en, end) - max(st, end - tail_ms)
            if ov > 0:
                agg[key(r["Kernel_Name"])] += ov
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:12]:
            print(f"  {v:7.2f} ms in the last {tail_ms:.0f} ms  {k}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 20.0)
