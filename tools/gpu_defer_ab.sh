# CCBAM input gradient formed inside the forked CBN backward (SEHIP_CCBAM_DEFER_DX=1, ABI 11)
# against the written form (=0): the CCBAM / CBN / FRCRN parity tests, then bench steps
# alternating the two.   gpurun -- bash tools/gpu_defer_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-defer}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_gpu_ccbam.py \
  $R/tests/test_gpu_cbn.py "$R/tests/test_gpu_models.py::test_frcrn_train_step_golden" \
  "$R/tests/test_gpu_models.py::test_train_step_deferred_weight_grads_bit_identical" > $O/tests.log 2>&1 \
  || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for d in 1 0 1 0; do
  SEHIP_CCBAM_DEFER_DX=$d timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/bench_$d.json 2> $O/bench_$d.err || exit 1
  python3 -c "
import json; d = json.loads(open('$O/bench_$d.json').read().strip().splitlines()[-1]); ob = d['op_breakdown']
print('defer=$d', d['value'], 'utt/s', {k: ob[k]['ms_per_step'] for k in ('ccbam_bwd', 'cbn_bwd', 'conv_data_joined_f16x3')})"
done
