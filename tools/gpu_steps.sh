# Per-step times with and without the CL16 copies: gpurun -- bash tools/gpu_steps.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-steps}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/step_times.py 14 > $O/on.log 2>&1 || exit $?
SEHIP_CL16=0 timeout -k 10 200 python3 $R/tools/step_times.py 14 > $O/off.log 2>&1 || exit $?
cat $O/on.log $O/off.log
