# Standalone GEMM pass profile (tools/conv_micro.py at FRCRN B=64 shapes):
# kernel trace, SQ counters, HBM traffic. Each GPU step has its own limit.
#   gpurun --timeout 900 -- bash tools/gpu_gemm_prof.sh <tag> [layers] [math]
R=$GRAFT_REPO_ROOT
TAG=${1:-gemm}; LAYERS=${2:-enc1,dec5}; MATH=${3:-f16x3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
M="$R/tools/conv_micro.py --layers $LAYERS --passes fwd,data,weight --math $MATH"
timeout -k 10 200 python3 $M --iters 5 > $O/micro.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $M --iters 3 > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- python3 $M --iters 1 > $O/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $M --iters 1 > $O/sq2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $O/tcc -o run --output-format csv -- python3 $M --iters 1 > $O/tcc.log 2>&1 || exit $?
echo done > $O/ok
