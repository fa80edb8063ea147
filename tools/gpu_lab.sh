# GEMM schedule lab (tools/gemm_lab.hip, built into tools/bin/gemm_lab on the CPU side):
#   gpurun -- bash tools/gpu_lab.sh <tag> [args...]
# timing run, then one SQ / GRBM counter pass (MFMA busy, effective clock, wait / issue split)
R=$GRAFT_REPO_ROOT; TAG=${1:-lab}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/bin/gemm_lab "$@" > $O/lab.log 2>&1 || { cat $O/lab.log; exit 1; }
cat $O/lab.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq --output-format csv -- $R/tools/bin/gemm_lab ${1:-4074496} 2 > $O/sq.log 2>&1 || exit 1
F=$(ls $O/sq/*counter_collection.csv $O/sq/*/*counter_collection.csv 2>/dev/null | head -1)
python3 $R/tools/sq_summary.py $F lab_v | tee $O/sq_summary.txt
