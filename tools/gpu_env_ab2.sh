# Selected GPU tests, then a same-box bench A/B of one env knob (off value vs default), twice:
#   gpurun -- bash tools/gpu_env_ab2.sh <tag> <VAR> <off-value> "<test paths>"
R=$GRAFT_REPO_ROOT; T=$1; V=$2; OFF=$3; TESTS=$4; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  P=""; for t in $TESTS; do P="$P $R/$t"; done
  timeout -k 10 500 python3 -u -m pytest $P -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
fi
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
for i in 1 2; do
  env $V=$OFF timeout -k 10 200 python3 $B > $O/bench_off$i.json 2> $O/bench_off$i.err || exit $?
  timeout -k 10 200 python3 $B > $O/bench_on$i.json 2> $O/bench_on$i.err || exit $?
done
echo ok > $O/ok
