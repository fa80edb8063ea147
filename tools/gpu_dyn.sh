# Dynamic-range tests of the f16x3 arithmetic (+ extra test files):
#   gpurun -- bash tools/gpu_dyn.sh <tag> [more test paths]
R=$GRAFT_REPO_ROOT
TAG=${1:-dyn}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="$R/tests/test_gpu_dynamic_range.py"
for t in "$@"; do ARGS="$ARGS $R/$t"; done
timeout -k 10 1000 python3 -u -m pytest $ARGS -v -s -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
exit $rc
