# Full GPU suite + a quick bench line + the STFT micro: gpurun --timeout 900 -- bash tools/gpu_full.sh <tag> [bench args]
R=$GRAFT_REPO_ROOT
TAG=${1:-full}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest $R/tests -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --compare "" "$@" > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 120 python3 $R/tools/stft_micro.py > $O/stft_micro.log 2>&1 || exit $?
exit $rc
