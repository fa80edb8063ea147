# Kernel-trace summaries of a short bench under two settings of one env knob:
# gpurun -- bash tools/gpu_ktrace_ab.sh <tag> <VAR> <off-value>
R=$GRAFT_REPO_ROOT; T=${1:-kt}; V=$2; OFF=$3; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/on -o run -- python3 $B > $O/on.log 2>&1 || exit $?
env $V=$OFF timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/off -o run -- python3 $B > $O/off.log 2>&1 || exit $?
echo ok > $O/ok
