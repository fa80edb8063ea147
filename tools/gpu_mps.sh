# Weight-grad m-split length A/B (SEHIP_WGRAD_MPS): micro timing + FETCH_SIZE per launch, then bench.
#   gpurun --timeout 900 -- bash tools/gpu_mps.sh <tag> <mps values...>
R=$GRAFT_REPO_ROOT
TAG=${1:-mps}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 "$@"; do
  echo "== MPS=$v" >> $O/mps.log
  SEHIP_WGRAD_MPS=$v timeout -k 10 120 python3 $R/tools/conv_micro.py --layers dec5,enc1 --passes weight --math f16x3 >> $O/mps.log 2>&1 || exit $?
  SEHIP_WGRAD_MPS=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$v -o run --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5,enc1 --passes weight --math f16x3 --iters 1 > $O/pmc_$v.log 2>&1 || exit $?
done
echo done > $O/ok
