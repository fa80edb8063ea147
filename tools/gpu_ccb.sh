# CCBAM fused sigmoid backward: CCBAM tests + model tests, then a same-box bench A/B against
# the previous library build (SEHIP_LIB): gpurun -- bash tools/gpu_ccb.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-ccb}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest $R/tests/test_gpu_ccbam.py $R/tests/test_gpu_models.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
for i in 1 2; do
timeout -k 10 200 python3 $B > $O/bench_on$i.json 2> $O/bench_on$i.err || exit $?
done
echo ok > $O/ok
