# SQ counters of the ConvSTFT / iSTFT kernels (stft_micro, two PMC passes + a kernel trace):
#   gpurun --timeout 600 -- bash tools/pmc_stft.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc_stft}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/stft_micro.py > $O/micro.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/stft_micro.py > $O/kt.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq1 -o run --output-format csv -- python3 $R/tools/stft_micro.py > $O/sq1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM -d $O/sq2 -o run --output-format csv -- python3 $R/tools/stft_micro.py > $O/sq2.log 2>&1 || exit $?
echo done > $O/ok
