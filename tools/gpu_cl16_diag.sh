# Kernel traces of the bench step with and without the CL16 weight-grad operands:
#   gpurun --timeout 900 -- bash tools/gpu_cl16_diag.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-cl16diag}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-op-timing --no-compare"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/on -o run -- python3 $B > $O/on.log 2>&1 || exit $?
export SEHIP_CL16=0
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/off -o run -- python3 $B > $O/off.log 2>&1 || exit $?
echo done > $O/ok
