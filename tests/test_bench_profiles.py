"""bench.py reads per-kernel figures from the committed profiles (rocprof kernel stats for
`rocprof_avg_ms_per_launch`, PMC traffic for `roofline.traffic`), keyed by kernel
instantiation: every instantiation its roofline table names must be present in both files,
so a renamed or re-templated kernel cannot silently turn those fields into null."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_kernels_are_in_the_committed_profiles():
    b = _bench()
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    with open(b.PROFILE_STATS) as f:
        stats = {b._kernel_key(r["Name"]) for r in csv.DictReader(f)}
    names = [b.KERNEL_OF[t][0] for t in ("conv_data_joined_f16x3", "conv_fwd_joined_f16x3",
                                         "conv_wgrad_joined_f16x3")]
    names += [k for _, k in b.STFT_KERNELS]
    for n in names:
        assert n in pmc, n
        assert n in stats or any(s.split("<")[0] == n for s in stats), n
