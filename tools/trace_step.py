"""Per-stream breakdown of one training step from a rocprofv3 kernel trace:
   python tools/trace_step.py <run_kernel_trace.csv> [step index from the end, default 1]"""
import collections
import csv
import re
import sys


def key(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    if n.startswith("Cijk"):
        return "rocBLAS " + n[:20]
    if n.startswith("at::") or "at::native" in n[:40]:
        m = re.search(r"at::native::(?:\w+::)*?(\w+(?:_kernel|Functor)\w*)", n)
        return "aten " + (m.group(1) if m else n[:40])
    return n.split("(")[0][:90]


if __name__ == "__main__":
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
    a, b = idx[-1 - back] + 1, idx[-back] + 1
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    print(f"step span {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")




    by = collections.defaultdict(list)
    for r in step:
        by[r["Stream_Id"]].append(r)
    for s, rs in sorted(by.items()):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e6
        gaps = 0
        for p, q in zip(rs, rs[1:]):
            gaps += max(0, int(q["Start_Timestamp"]) - int(p["End_Timestamp"]))
        print(f"\n== stream {s}: {len(rs)} kernels, busy {busy:.1f} ms, gaps {gaps / 1e6:.1f} ms")
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in rs:
            k = key(r["Kernel_Name"])
            agg[k][0] += 1
            agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
            print(f"{d / 1e3:7.2f} ms {n:4d}  {k}")
