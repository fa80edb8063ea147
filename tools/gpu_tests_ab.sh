# Selected GPU tests, then a same-box A/B of env knobs on the default bench step
# (two rounds of each config, short bench):
#   gpurun --timeout 1200 -- bash tools/gpu_tests_ab.sh <tag> "<test paths>" "ENV=a" "ENV=b" ...
R=$GRAFT_REPO_ROOT
TAG=$1; TESTS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=""
for t in $TESTS; do ARGS="$ARGS $R/$t"; done
if [ -n "$ARGS" ]; then
  timeout -k 10 480 python3 -u -m pytest $ARGS -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for rep in 1 2; do
  i=0
  for cfg in "" "$@"; do
    env $cfg timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-op-timing --no-compare > $O/ab_${i}_$rep.json 2>> $O/ab.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/ab_${i}_$rep.json').read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'])" >> $O/ab.log
    i=$((i+1))
  done
done
echo done > $O/ok
