# Bench runs separated by the given sleeps (seconds): does a process's step rate depend on
# how long ago the previous GPU process ended?
#   gpurun -- bash tools/gpu_gap.sh <tag> "0 45 0 90"
R=$GRAFT_REPO_ROOT
TAG=${1:-gap}
O=$R/gpurun_out/$TAG
mkdir -p $O
B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
n=0
for s in $2; do
  n=$((n + 1))
  sleep $s
  timeout -k 10 240 $B > $O/run$n.json 2> $O/run$n.err || exit $?
  echo "sleep $s: $(grep -h 'utt/s' $O/run$n.err)"
done
