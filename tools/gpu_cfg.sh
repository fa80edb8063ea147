# Config tests + configs bench: gpurun --timeout 900 -- bash tools/gpu_cfg.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-cfg}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_longform.py -v -s -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python3 $R/tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit $?
echo done > $O/ok
