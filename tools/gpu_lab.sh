# GEMM schedule lab (tools/gemm_lab.hip, built into tools/bin/gemm_lab on the CPU side):
#   gpurun -- bash tools/gpu_lab.sh <tag> [args...]
R=$GRAFT_REPO_ROOT; TAG=${1:-lab}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/bin/gemm_lab "$@" > $O/lab.log 2>&1; rc=$?
cat $O/lab.log; exit $rc
