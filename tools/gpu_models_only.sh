# model parity tests only
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-mo}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_models.py -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo ok > $O/ok
