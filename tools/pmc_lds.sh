# LDS bank-conflict rate of the conv GEMM passes (conv_micro, one PMC pass):
#   gpurun --timeout 600 -- bash tools/pmc_lds.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc_lds}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/lds --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5,enc1 --passes fwd,data,weight --math f16x3 --iters 1 > $O/lds.log 2>&1 || exit $?
echo done > $O/ok
