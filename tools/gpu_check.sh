# Full GPU test suite, then one bench line (no CPU baseline). A test failure
# (rc 1) does not stop the script; a crash, abort or timeout does.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag> [bench args...]
R=$GRAFT_REPO_ROOT
TAG=${1:-check}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 python3 -u -m pytest $R/tests -v -s -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || exit $?
echo done > $O/ok
