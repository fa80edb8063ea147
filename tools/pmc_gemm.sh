# SQ stall breakdown of the conv GEMM passes (conv_micro, one PMC pass):
#   gpurun --timeout 600 -- bash tools/pmc_gemm.sh <tag> [conv_micro args]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc_sq}; shift || true
ARGS=${@:---layers dec5,enc1 --passes fwd,data,weight --math f16x3 --iters 1}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq --output-format csv -- python3 $R/tools/conv_micro.py $ARGS > $O/sq.log 2>&1
echo done > $O/ok
