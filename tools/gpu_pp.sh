# Ping-pong gather (SEHIP_GEMM_PP=1): bit-identity vs the default schedule, micro timing, bench A/B.
R=$GRAFT_REPO_ROOT
TAG=${1:-pp}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/bm_check.py $O/a.pt > $O/check.log 2>&1 || exit $?
SEHIP_GEMM_PP=2 timeout -k 10 120 python3 $R/tools/bm_check.py $O/b.pt >> $O/check.log 2>&1 || exit $?
python3 -c "import torch; a=torch.load('$O/a.pt'); b=torch.load('$O/b.pt'); print({k: bool(torch.equal(a[k], b[k])) for k in a})" >> $O/check.log 2>&1
rm -f $O/*.pt
timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 > $O/micro_def.log 2>&1 || exit $?
SEHIP_GEMM_PP=1 timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 > $O/micro_pp.log 2>&1 || exit $?
SEHIP_GEMM_PP=2 timeout -k 10 200 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 > $O/micro_pp2.log 2>&1 || exit $?
bash $R/tools/gpu_ab.sh $TAG "SEHIP_GEMM_PP=2"
