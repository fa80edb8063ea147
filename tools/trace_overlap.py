"""What runs beside the kernels matching a substring, in one training step of a
rocprofv3 kernel trace: python tools/trace_overlap.py <trace.csv> <substring> [step from the end]"""
import csv
import sys

from trace_step import key   # noqa: E402  (same directory)

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sub = sys.argv[2]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
step = rows[idx[-1 - back] + 1: idx[-back] + 1]
t0 = int(step[0]["Start_Timestamp"])
for r in step:
    if sub not in r["Kernel_Name"]:
        continue
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"\n{key(r['Kernel_Name'])} stream {r['Stream_Id']} at {(a - t0) / 1e6:.2f} ms, {(b - a) / 1e3:.0f} us")
    for q in step:
        qa, qb = int(q["Start_Timestamp"]), int(q["End_Timestamp"])
        ov = min(b, qb) - max(a, qa)
        if q is not r and ov > 0:
            print(f"   {ov / 1e3:8.0f} us  s{q['Stream_Id']}  {key(q['Kernel_Name'])}")
