# Configs (default 2 and 3: DCUNet-16 bf16 inference, DCCRN-CL bf16 train; 5: CARN fp16
# 30 s @ 48 kHz) timed, then each under rocprofv3 --kernel-trace --stats, then the two PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE) of each, summarised per kernel instantiation:
#   gpurun -- bash tools/gpu_cfg_prof.sh <tag> [configs, e.g. 3,5] [pmc: 1|0]
R=$GRAFT_REPO_ROOT
TAG=${1:-cfgprof}
CFGS=${2:-2,3}
PMC=${3:-1}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/tools/bench_configs.py --configs $CFGS --iters 10 > $O/configs.jsonl 2> $O/configs.err || exit $?
for c in ${CFGS//,/ }; do
  ST=bf16; [ "$c" = 5 ] && ST=fp16
  # whole program + the timed iterations' roctx range (tools/region_stats.py filters by it)
  SEHIP_ROCTX_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof$c -o run -- python3 $R/tools/bench_configs.py --configs $c --storage $ST --iters 5 > $O/prof$c.log 2>&1 || exit $?
  python3 $R/tools/region_stats.py $O/prof$c $O/config${c}_region_kernel_stats.csv >> $O/region_stats.log 2>&1 || exit $?
  [ "$PMC" = 1 ] || continue
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc${c}_fetch -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs $c --storage $ST --iters 1 > $O/pmc${c}_fetch.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc${c}_write -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs $c --storage $ST --iters 1 > $O/pmc${c}_write.log 2>&1 || exit $?
  python3 $R/tools/pmc_summary.py $O/pmc${c}_fetch $O/pmc${c}_write $O/pmc${c}_traffic.json > $O/pmc${c}_summary.log 2>&1 || exit $?
done
echo ok > $O/ok
