"""Kernel statistics of the timed region only: the kernels of a rocprofv3 --kernel-trace
--marker-trace run whose execution starts inside a roctx range named "timed" (bench.py /
tools/bench_configs.py with SEHIP_ROCTX_REGIONS=1 push it after the warm-up's synchronize
and pop it after the timed loop's). Written in the column layout of rocprofv3's
kernel_stats.csv, so bench.py's readers and tools/aten_sources.py take either.

  python tools/region_stats.py <rocprofv3 output dir> <out.csv> [range name, default timed]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _one(d, pat):
    fs = sorted(glob.glob(os.path.join(d, pat)) + glob.glob(os.path.join(d, "*", pat)))
    if not fs:
        raise SystemExit(f"region_stats: no {pat} under {d}")
    return fs[0]


def ranges(marker_csv, name):
    out = []
    with open(marker_csv) as f:
        for r in csv.DictReader(f):
            label = r.get("Message") or r.get("Name") or r.get("Function") or ""
            if label == name or label.endswith(name):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def main():
    d, out_csv = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else "timed"
    rg = ranges(_one(d, "*marker_api_trace.csv"), name)
    if not rg:
        raise SystemExit(f"region_stats: no roctx range {name!r} in {d}")
    durs = defaultdict(list)
    with open(_one(d, "*kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if any(a <= s <= b for a, b in rg):
                durs[r["Kernel_Name"]].append(e - s)
    total = sum(sum(v) for v in durs.values()) or 1
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    print(f"{len(rg)} range(s) {name!r}: {sum(len(v) for v in durs.values())} kernels, "
          f"{len(durs)} names, {total / 1e6:.2f} ms -> {out_csv}")


if __name__ == "__main__":
    main()
