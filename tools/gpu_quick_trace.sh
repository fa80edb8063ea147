# Selected tests, then a kernel-trace summary of a short bench: gpurun -- bash tools/gpu_quick_trace.sh <tag> "<tests>"
R=$GRAFT_REPO_ROOT; T=$1; TESTS=$2; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  P=""; for t in $TESTS; do P="$P $R/$t"; done
  timeout -k 10 500 python3 -u -m pytest $P -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare > $O/prof_bench.log 2>&1 || exit $?
echo ok > $O/ok
