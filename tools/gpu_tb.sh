# Selected GPU tests, then (if they pass) a short bench line:
#   gpurun --timeout 900 -- bash tools/gpu_tb.sh <tag> <test paths...>
R=$GRAFT_REPO_ROOT
TAG=${1:-tb}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=""
for t in "$@"; do ARGS="$ARGS $R/$t"; done
timeout -k 10 600 python3 -u -m pytest $ARGS -v -s -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --compare "" > $O/bench.json 2> $O/bench.err || exit $?
exit $rc
