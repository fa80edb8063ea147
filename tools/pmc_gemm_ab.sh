# SQ stall breakdown of one conv GEMM pass, default library vs variant libraries:
#   gpurun --timeout 600 -- bash tools/pmc_gemm_ab.sh <tag> "<conv_micro args>" <variants...>
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc_ab}; ARGS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/def --output-format csv -- python3 $R/tools/conv_micro.py $ARGS > $O/def.log 2>&1 || exit $?
for v in "$@"; do
  SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/$v --output-format csv -- python3 $R/tools/conv_micro.py $ARGS > $O/$v.log 2>&1 || exit $?
done
echo done > $O/ok
