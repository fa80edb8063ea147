# CBN micro (tools/cbn_micro.py) A/B between the in-tree library and variant builds,
# alternating, after the CBN GPU tests on the in-tree library:
#   gpurun -- bash tools/gpu_cbn_ab.sh <tag> <variant> [<variant> ...]
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_gpu_cbn.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  echo "== round $r cur" >> $O/ab.log
  timeout -k 10 200 python3 $R/tools/cbn_micro.py >> $O/ab.log 2>&1 || exit $?
  for V in "$@"; do
    echo "== round $r $V" >> $O/ab.log
    SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so timeout -k 10 200 python3 $R/tools/cbn_micro.py >> $O/ab.log 2>&1 || exit $?
  done
done
cat $O/ab.log
