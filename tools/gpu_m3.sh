# 3M forward: its tests, then the model / dynamic-range suites with SEHIP_GEMM_3M=1, then a
# same-box bench A/B: gpurun -- bash tools/gpu_m3.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-m3}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_conv_3m.py -v -s --timeout 250 --timeout-method thread -p no:cacheprovider > $O/tests_3m.log 2>&1 || exit $?
SEHIP_GEMM_3M=1 timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_models.py $R/tests/test_gpu_dynamic_range.py $R/tests/test_gpu_longform.py -v --timeout 500 --timeout-method thread -p no:cacheprovider > $O/tests_models_3m.log 2>&1
echo "rc=$?" >> $O/tests_models_3m.log
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
for i in 1 2; do
  SEHIP_GEMM_3M=1 timeout -k 10 200 python3 $B > $O/bench_3m$i.json 2> $O/bench_3m$i.err || exit $?
  timeout -k 10 200 python3 $B > $O/bench_4m$i.json 2> $O/bench_4m$i.err || exit $?
done
echo ok > $O/ok
