# Weight-grad m-split size: PMC traffic per instantiation and a same-box bench A/B per
# SEHIP_WGRAD_MPS value: gpurun -- bash tools/gpu_mps.sh <tag> <mps values...>
R=$GRAFT_REPO_ROOT; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B1="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare"
for v in "$@"; do
  SEHIP_WGRAD_MPS=$v timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$v -o run --output-format csv -- python3 $B1 > $O/f$v.log 2>&1 || exit $?
  SEHIP_WGRAD_MPS=$v timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$v -o run --output-format csv -- python3 $B1 > $O/w$v.log 2>&1 || exit $?
  python3 $R/tools/pmc_summary.py $O/f$v $O/w$v $O/pmc_$v.json > $O/pmc_$v.log 2>&1 || exit $?
done
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
for i in 1 2; do
  for v in "$@"; do
    SEHIP_WGRAD_MPS=$v timeout -k 10 200 python3 $B > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit $?
  done
done
echo ok > $O/ok
