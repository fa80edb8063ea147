# One gpurun call: GPU parity tests, the default bench line (with CPU
# baseline), a rocprofv3 kernel-trace summary of a short bench, and the two PMC
# passes (FETCH_SIZE / WRITE_SIZE, separate runs) behind profiles/pmc_traffic.json.
# A test failure (rc 1) does not stop the script; a crash, abort or timeout ends it.
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> [pytest selection]
R=$GRAFT_REPO_ROOT
TAG=${1:-run}
SEL=${2:-tests}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 python3 -u -m pytest $R/$SEL -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 420 python3 $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare > $O/prof_bench.log 2>&1 || exit $?
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
python3 $R/tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json > $O/pmc_summary.log 2>&1
echo done > $O/ok
