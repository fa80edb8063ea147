# Final-tree check: smoke + the full GPU suite: gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-final}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp
timeout -k 10 800 python3 -u -m pytest $R/tests -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
echo ok > $O/ok
exit $rc
