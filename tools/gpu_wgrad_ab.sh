# Encoder weight-grad 256 x 128 tiles (default) vs 128 x 128 (SEHIP_WGRAD_K256=0): conv tests,
# conv_micro weight-grad timings, bench steps alternating, and the PMC traffic of one step each.
#   gpurun -- bash tools/gpu_wgrad_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-wgk}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $R/tests/test_gpu_conv_x3.py \
  "$R/tests/test_gpu_models.py::test_frcrn_train_step_golden" > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for k in 1 0 1 0; do
  SEHIP_WGRAD_K256=$k timeout -k 10 120 python3 $R/tools/conv_micro.py --layers enc1,enc4 --passes weight --math f16x3 --iters 10 > $O/micro_$k.log 2>&1 || exit 1
  echo "k256=$k $(grep -h weight $O/micro_$k.log | tr '\n' ' ')"
done
for k in 1 0 1 0; do
  SEHIP_WGRAD_K256=$k timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/bench_$k.json 2> $O/bench_$k.err || exit 1
  python3 -c "
import json; d = json.loads(open('$O/bench_$k.json').read().strip().splitlines()[-1]); ob = d['op_breakdown']
print('k256=$k', d['value'], 'utt/s', {x: ob[x]['ms_per_step'] for x in ('conv_wgrad_f16x3', 'conv_wgrad_joined_f16x3', 'conv_data_joined_f16x3')})"
done
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
python3 $R/tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json > $O/pmc_summary.log 2>&1 || exit $?
grep -h "wgrad" $O/pmc_summary.log | head -n 8
