# Configs 2 and 3 (DCUNet-16 bf16 inference, DCCRN-CL bf16 train) timed, then each under
# rocprofv3 --kernel-trace --stats: gpurun -- bash tools/gpu_cfg_prof.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-cfgprof}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/bench_configs.py --configs 2,3 --iters 10 > $O/configs.jsonl 2> $O/configs.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 $R/tools/bench_configs.py --configs 2 --iters 5 > $O/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 $R/tools/bench_configs.py --configs 3 --iters 5 > $O/prof3.log 2>&1 || exit $?
echo ok > $O/ok
