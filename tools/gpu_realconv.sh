set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-rc}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_cconv.py -v -m gpu -k real_conv_geometries --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || true
echo ok > $O/ok
