# smoke + full GPU suite + configs 2/3/5 timing (after the round-3 changes)
R=$GRAFT_REPO_ROOT; T=${1:-chk6}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp
timeout -k 10 700 python3 -u -m pytest $R/tests -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/tools/bench_configs.py --configs 2,3,5 --iters 10 > $O/configs.jsonl 2> $O/configs.err || exit $?
