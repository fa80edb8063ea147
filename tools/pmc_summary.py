"""Turn rocprofv3 PMC passes into per-launch HBM traffic for bench.py.

Usage: python tools/pmc_summary.py <fetch_dir> <write_dir> [out.json]
Each dir holds a rocprofv3 --pmc csv run (run_counter_collection.csv) of the
same bench command, one with FETCH_SIZE, one with WRITE_SIZE (TCC slots do not
fit both in one pass). gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE counts 64 B per 128-B request of wide streaming reads, i.e. half the
bytes -> doubled; both counters are in KiB.
"""
import collections, csv, json, os, re, sys


def kernel_key(name):
    """rocprof kernel name -> 'base<template args>' (as bench.py's _kernel_key)."""
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void\s+", "", name)
    depth, end = 0, len(name)
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            end = i
            break
    name = name[:end].strip()
    return name if "<" in name else name.split("::")[-1].strip()


def load(d, counter):
    """Per kernel: values of every dispatch, keyed by the exact instantiation and,
    aggregated, by the base name."""
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):   # rocprofv3 -d without -o: <d>/<host>/<pid>_counter_collection.csv
        import glob
        path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[-1]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        full = kernel_key(r["Kernel_Name"])
        v = float(r["Counter_Value"]) * 1024.0
        per[full].append(v)
        base = full.split("<")[0].split("::")[-1].strip()
        if base != full:
            per[base].append(v)
    return per


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        if not f or not w:
            continue
        fb = 2.0 * sum(f) / len(f)          # gfx950: FETCH_SIZE reads half the streamed bytes
        wb = sum(w) / len(w)
        res[k] = {"launches": len(f), "fetch_bytes_per_launch_corrected": fb,
                  "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k in ("gather_x3_kernel<true, 3, 2, 2, true, 0>", "wgrad_x3_kernel<true, 3, true, true, 2, false, 0, 2>",
              "stft_fwd_rg_kernel", "istft_fwd_wv_kernel", "istft_bwd_rg_kernel", "cbn_apply_kernel"):
        if k in res:
            print(k, {a: f"{b:.4g}" for a, b in res[k].items()})


if __name__ == "__main__":
    main()
