# bit-identity vs the previous library (CBN apply load batching), the channel-blocked first-block
# backward tests, then a same-box A/B: current, previous library, SEHIP_FC_CPB=2, =4
R=$GRAFT_REPO_ROOT; T=${1:-fix8}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
PREV=$R/speech-enhancement_amd/sehip/libsehip_prev.so
SEHIP_LIB=$PREV timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_prev.pt || exit $?
timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_cur.pt || exit $?
python3 $R/tools/grads_dump.py cmp /tmp/g_prev.pt /tmp/g_cur.pt > $O/cmp.log 2>&1
timeout -k 10 400 python3 -u -m pytest -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
  $R/tests/test_gpu_cbn.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash $R/tools/gpu_tests_ab.sh $T/ab "" "SEHIP_LIB=$PREV" "SEHIP_FC_CPB=2" "SEHIP_FC_CPB=4"
