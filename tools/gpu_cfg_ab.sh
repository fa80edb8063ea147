# Configs 2/3 (tools/bench_configs.py, bf16 storage) alternating between the in-tree library
# and variant builds, two rounds:  gpurun -- bash tools/gpu_cfg_ab.sh <tag> <variant> [...]
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python3 $R/tools/bench_configs.py --configs 2,3 --storage bf16 --iters 10 > $O/cur_$r.jsonl 2>&1 || exit $?
  for V in "$@"; do
    SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so timeout -k 10 300 python3 $R/tools/bench_configs.py --configs 2,3 --storage bf16 --iters 10 > $O/${V}_$r.jsonl 2>&1 || exit $?
  done
done
for f in $O/*.jsonl; do echo "== $(basename $f)"; grep -h '"config"' $f | python3 -c "import sys,json; [print(d['config'], d['storage'], d['value'], d['roofline']['frac']) for d in map(json.loads, sys.stdin)]"; done
