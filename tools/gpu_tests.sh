# Selected GPU tests only: gpurun --timeout 600 -- bash tools/gpu_tests.sh <tag> <test paths...>
R=$GRAFT_REPO_ROOT
TAG=${1:-t}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=""
for t in "$@"; do ARGS="$ARGS $R/$t"; done
timeout -k 10 480 python3 -u -m pytest $ARGS -v -s -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
exit $rc
