# gpurun --timeout 300 -- bash tools/gpu_stencil_debug.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-stcdbg}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_stcdbg.so timeout -k 10 120 python3 $R/tools/stencil_debug.py > $O/out.log 2>&1
rc=$?; cat $O/out.log; exit $rc
