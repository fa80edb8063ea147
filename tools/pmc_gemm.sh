set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5 --passes fwd,data,weight --math bf16x3,bf16x6 --iters 1 > $R/gpurun_out/pmc_sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $R/gpurun_out/pmc_tcc --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5 --passes fwd,data,weight --math bf16x3,bf16x6 --iters 1 > $R/gpurun_out/pmc_tcc.log 2>&1
