# Alternating A/B of the ConvSTFT / iSTFT micro (tools/stft_micro.py) between the
# in-tree library and variant builds (make variant V=name), three rounds:
#   gpurun -- bash tools/gpu_stft_ab.sh <tag> <variant> [<variant> ...]
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in 1 2 3; do
  echo "== round $r cur" | tee -a $O/ab.log
  timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/ab.log 2>&1 || exit $?
  for V in "$@"; do
    echo "== round $r $V" | tee -a $O/ab.log
    SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/ab.log 2>&1 || exit $?
  done
done
cat $O/ab.log
