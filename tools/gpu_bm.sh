# SEHIP_GEMM_BM A/B: bit-identity of the 256-row tiles vs the 128-row ones, micro timing, bench.
#   gpurun --timeout 900 -- bash tools/gpu_bm.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-bm}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/bm_check.py $O/bm128.pt > $O/check.log 2>&1 || exit $?
SEHIP_GEMM_BM=256 timeout -k 10 120 python3 $R/tools/bm_check.py $O/bm256.pt >> $O/check.log 2>&1 || exit $?
python3 -c "import torch; a=torch.load('$O/bm128.pt'); b=torch.load('$O/bm256.pt'); print({k: bool(torch.equal(a[k], b[k])) for k in a})" >> $O/check.log 2>&1
rm -f $O/*.pt
timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 > $O/micro128.log 2>&1 || exit $?
SEHIP_GEMM_BM=256 timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 > $O/micro256.log 2>&1 || exit $?
bash $R/tools/gpu_ab.sh $TAG "SEHIP_GEMM_BM=256"
