# Packed gather GEMM 256x256 two-stage variant (SEHIP_GEMM_BM=256) vs the 128x256 three-stage one.
R=$GRAFT_REPO_ROOT
TAG=${1:-pk256}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 --packed > $O/bm128.log 2>&1 || exit $?
SEHIP_GEMM_BM=256 timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 --packed > $O/bm256.log 2>&1 || exit $?
SEHIP_GEMM_BM=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 --packed --iters 3 > $O/trace.log 2>&1 || exit $?
echo done > $O/ok
