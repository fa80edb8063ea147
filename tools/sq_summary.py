"""Summarise a rocprofv3 SQ counter pass (tools/pmc_gemm.sh) per GEMM kernel.

MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs), with
cycles = GRBM_GUI_ACTIVE / 8: rocprofv3 reports GRBM_GUI_ACTIVE summed over the
8 XCDs (MI355X_MICROARCH.md, DVFS give-back). SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles.
Usage: python tools/sq_summary.py <counter_collection.csv> [kernel-name substring, default x3_kernel]
"""
import csv
import re
import sys
from collections import defaultdict

rows = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
dur = defaultdict(dict)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        k = r["Kernel_Name"]
        if (sys.argv[2] if len(sys.argv) > 2 else "x3_kernel") not in k:
            continue
        mk = re.search(r"\w+_kernel<[^>]*>", k) or re.search(r"\w+<[^>]*>|\w+", k)
        k = mk.group(0)
        rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for k, c in rows.items():
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    wall = sum(dur[k].values())
    print(f"{k} dispatches {len(disp[k])}")
    print(f"   MFMA busy / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) = {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f} ; "
          f"effective clock GRBM_GUI_ACTIVE / 8 / wall = {cyc / wall / 1e9:.2f} GHz (profiled)")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        print(f"   of wave cycles: waiting (s_waitcnt / barrier) {c['SQ_WAIT_ANY'] / wc:.3f}, issue-stalled "
              f"{c['SQ_WAIT_INST_ANY'] / wc:.3f} (LDS issue {c.get('SQ_WAIT_INST_LDS', 0) / wc:.3f}), "
              f"issuing {c['SQ_ACTIVE_INST_ANY'] / wc:.3f}")
