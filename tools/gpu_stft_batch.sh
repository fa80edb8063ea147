# ConvSTFT / iSTFT per-launch time against the batch (tools/stft_micro.py, STFT_B=n), for
# the in-tree library and variant builds: gpurun -- bash tools/gpu_stft_batch.sh <tag> [variant ...]
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for V in cur "$@"; do
  L=$R/speech-enhancement_amd/sehip/libsehip.so
  [ $V != cur ] && L=$R/speech-enhancement_amd/sehip/libsehip_$V.so
  for b in 32 48 56 60 62 64 66 72 80 96 112 128; do
    echo "$V B=$b" >> $O/batch.log
    SEHIP_LIB=$L STFT_B=$b timeout -k 10 100 python3 $R/tools/stft_micro.py >> $O/batch.log 2>&1 || exit $?
  done
done
cat $O/batch.log
