"""Main-stream kernels of one training step from a rocprofv3 kernel trace, each with its
duration and the side-stream kernels that overlap it (to see which short launches stretch
while the weight-grads hold the CUs):
   python tools/trace_stalls.py <run_kernel_trace.csv> [name filter] [step index from the end]"""
import csv
import sys

from trace_step import key

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
step = rows[idx[-1 - back] + 1: idx[-back] + 1]
streams = sorted({r["Stream_Id"] for r in step}, key=lambda s: -sum(1 for r in step if r["Stream_Id"] == s))
main = streams[0]
t0 = int(step[0]["Start_Timestamp"])
side = [r for r in step if r["Stream_Id"] != main]
tot = 0.0
for r in step:
    if r["Stream_Id"] != main or flt not in r["Kernel_Name"]:
        continue
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ov = [key(s["Kernel_Name"])[:40] for s in side if int(s["Start_Timestamp"]) < b and int(s["End_Timestamp"]) > a]
    tot += (b - a) / 1e3
    print(f"{(a - t0) / 1e3:9.1f} us {(b - a) / 1e3:8.1f} us  {key(r['Kernel_Name'])[:60]:60s} | {', '.join(sorted(set(ov)))}")
print(f"total {tot / 1e3:.2f} ms")
