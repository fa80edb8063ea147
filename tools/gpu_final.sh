# Round-end evidence on one box: the full GPU suite, smoke(), then tools/gpu_evidence.sh
# (kernel trace, PMC traffic, step trace summary, the default bench line with the CPU baseline):
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag> <round>
R=$GRAFT_REPO_ROOT; TAG=${1:-final}; RND=${2:-r5}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
(cd $R && timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()") > $O/smoke.log 2>&1 || exit $?
bash $R/tools/gpu_evidence.sh ${TAG}_ev $RND || exit $?
exit $rc
