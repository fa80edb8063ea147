# Kernel trace of a short default bench (optionally with env knobs):
#   gpurun --timeout 600 -- bash tools/gpu_prof_quick.sh <tag> [ENV=v ...]
R=$GRAFT_REPO_ROOT; TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare > $O/prof_bench.log 2>&1 || exit $?
echo ok > $O/ok
