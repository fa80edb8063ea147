# fused-head check: its parity tests + the model tests, then a same-box A/B of SEHIP_HEAD
#   gpurun --timeout 900 -- bash tools/gpu_head.sh <tag>
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_cbn.py $R/tests/test_gpu_models.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for rep in 1 2; do
  for v in 1 0; do
    env SEHIP_HEAD=$v timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-op-timing --no-compare > $O/head_${v}_$rep.json 2>> $O/bench.err
    python3 -c "import json; d=json.loads(open('$O/head_${v}_$rep.json').read().strip().splitlines()[-1]); print('SEHIP_HEAD=$v', d['value'], d['ms_per_step'])" >> $O/ab.log
  done
done
echo ok > $O/ok
