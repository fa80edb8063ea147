# rocprofv3 kernel-trace stats of a short bench run (profiles/ evidence).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare-f32 > $R/gpurun_out/prof_bench.log 2>&1
