# conv_micro on the GPU: gpurun --timeout 600 -- bash tools/gpu_micro.sh <tag> <conv_micro args...>
R=$GRAFT_REPO_ROOT
TAG=${1:-micro}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/conv_micro.py "$@" > $O/micro.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/conv_micro.py "$@" --iters 3 > $O/trace.log 2>&1 || exit $?
echo done > $O/ok
