# model parity tests + two bench lines (no CPU baseline / comparison steps)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-mb}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_models.py $R/tests/test_gpu_cbn.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --compare "" > $O/b1.json 2> $O/b1.err
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --compare "" > $O/b2.json 2> $O/b2.err
echo ok > $O/ok
