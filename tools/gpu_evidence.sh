# Round evidence in dependency order: kernel trace + the two PMC passes of a short bench,
# their summaries copied into this box's profiles/ (the files bench.py reads for
# rocprof_avg_ms_per_launch and roofline.traffic), then the default bench line (CPU baseline
# included) against them:  gpurun --timeout 1200 -- bash tools/gpu_evidence.sh <tag> <round, e.g. r4>
R=$GRAFT_REPO_ROOT; TAG=${1:-ev}; RND=${2:-r5}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
# whole program (the warm-up steps run the same kernels as the timed ones; the few data-
# generation kernels have their own names); --marker-trace records the timed steps' roctx
# range (SEHIP_ROCTX_REGIONS=1) for tools/region_stats.py
SEHIP_ROCTX_REGIONS=1 timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-op-timing --no-compare > $O/prof_bench.log 2>&1 || exit $?
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
python3 $R/tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json > $O/pmc_summary.log 2>&1 || exit $?
STATS=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1)
TRACE=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/trace_step.py $TRACE > $O/step_trace_summary.txt 2>&1 || exit $?
python3 $R/tools/region_stats.py $O/prof $O/region_kernel_stats.csv > $O/region_stats.log 2>&1 || exit $?
cp $O/region_kernel_stats.csv $R/profiles/${RND}_bench_kernel_stats.csv && cp $STATS $R/profiles/${RND}_bench_kernel_stats_whole_program.csv && cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json || exit 1
timeout -k 10 560 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo done > $O/ok
