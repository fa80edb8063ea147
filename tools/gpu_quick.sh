set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/g1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_cbn.py $R/tests/test_gpu_models.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-compare > $O/bench.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ccbam -o run -- python3 $R/tools/ccbam_micro.py > $O/ccbam.log 2>&1
echo ok > $O/ok
