# se_gemm LSTM GEMMs: new tests, the LSTM suites, then a same-box bench A/B
# (SEHIP_LSTM_GEMM=torch vs default): gpurun --timeout 900 -- bash tools/gpu_gemm.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-gemm}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_gemm.py $R/tests/test_gpu_lstm.py $R/tests/test_gpu_lstm_wide.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
SEHIP_LSTM_GEMM=torch timeout -k 10 200 python3 $B > $O/bench_off.json 2> $O/bench_off.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on.json 2> $O/bench_on.err || exit $?
SEHIP_LSTM_GEMM=torch timeout -k 10 200 python3 $B > $O/bench_off2.json 2> $O/bench_off2.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on2.json 2> $O/bench_on2.err || exit $?
echo ok > $O/ok
