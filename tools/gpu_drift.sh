# Is the FRCRN step rate a property of the process or of the GPU's state? Two bench runs
# back to back (a long one, then a short one), rocm-smi power / clocks sampled every
# second in the background meanwhile.
#   gpurun -- bash tools/gpu_drift.sh <tag> [steps of the first run]
R=$GRAFT_REPO_ROOT
TAG=${1:-drift}
S1=${2:-100}
O=$R/gpurun_out/$TAG
mkdir -p $O
B="python3 $R/bench.py --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
( for i in $(seq 1 150); do date +%T.%N; timeout -k 2 5 rocm-smi --showpower --showclocks --showuse 2>&1 | grep -E "Power|sclk|mclk|use"; sleep 1; done ) > $O/smi.log 2>&1 &
SMI=$!
timeout -k 10 240 $B --steps $S1 > $O/run1.json 2> $O/run1.err
rc=$?
[ $rc = 0 ] && { timeout -k 10 240 $B --steps 20 > $O/run2.json 2> $O/run2.err; rc=$?; }
[ $rc = 0 ] && { timeout -k 10 240 $B --steps 20 > $O/run3.json 2> $O/run3.err; rc=$?; }
kill $SMI
grep -h "utt/s" $O/run*.err
exit $rc
