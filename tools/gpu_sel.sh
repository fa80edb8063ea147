# Selected GPU tests (-s) + optional quick bench: gpurun -- bash tools/gpu_sel.sh <tag> "<pytest node ids>" [bench]
R=$GRAFT_REPO_ROOT
TAG=${1:-sel}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=""
for t in $2; do ARGS="$ARGS $R/$t"; done
timeout -k 10 600 python3 -u -m pytest $ARGS -v -s -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ "$3" = "bench" ]; then
  timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --compare "" > $O/bench.json 2> $O/bench.err || exit $?
fi
exit $rc
