# Forward-built data-grad weight images: new tests, a same-box bench A/B
# (SEHIP_DATA_PREP=0 vs default), the full GPU suite, then configs 2/3 profiled:
# gpurun --timeout 1200 -- bash tools/gpu_dw.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-dw}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest $R/tests/test_gpu_data_weights.py $R/tests/test_abi.py -v -m "gpu or not gpu" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/dw_tests.log 2>&1 || exit $?
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
SEHIP_DATA_PREP=0 timeout -k 10 200 python3 $B > $O/bench_off.json 2> $O/bench_off.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on.json 2> $O/bench_on.err || exit $?
SEHIP_DATA_PREP=0 timeout -k 10 200 python3 $B > $O/bench_off2.json 2> $O/bench_off2.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on2.json 2> $O/bench_on2.err || exit $?
timeout -k 10 500 python3 -u -m pytest $R/tests -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 $R/tools/bench_configs.py --configs 2 --iters 5 > $O/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 $R/tools/bench_configs.py --configs 3 --iters 5 > $O/prof3.log 2>&1 || exit $?
echo ok > $O/ok
exit $rc
