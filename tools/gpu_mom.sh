# CBN moments from the conv epilogue: new tests, a same-box bench A/B
# (SEHIP_CONV_MOMENTS=0 vs default), then the full GPU suite:
# gpurun --timeout 1200 -- bash tools/gpu_mom.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-mom}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_conv_moments.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/mom_tests.log 2>&1 || exit $?
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
SEHIP_CONV_MOMENTS=0 timeout -k 10 200 python3 $B > $O/bench_off.json 2> $O/bench_off.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on.json 2> $O/bench_on.err || exit $?
SEHIP_CONV_MOMENTS=0 timeout -k 10 200 python3 $B > $O/bench_off2.json 2> $O/bench_off2.err || exit $?
timeout -k 10 200 python3 $B > $O/bench_on2.json 2> $O/bench_on2.err || exit $?
timeout -k 10 500 python3 -u -m pytest $R/tests -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
echo ok > $O/ok
exit $rc
