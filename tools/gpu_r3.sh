# Round-3 evidence (tools/gpu_round.sh) followed by the STFT probe timings (tools/stft_probe.sh builds)
R=$GRAFT_REPO_ROOT; TAG=${1:-r3}
bash $R/tools/gpu_round.sh $TAG || exit $?
O=$R/gpurun_out/$TAG; cd /tmp && export TMPDIR=/tmp
for k in 0 1 2 3 0; do
  L=$R/speech-enhancement_amd/sehip/libsehip_stftp$k.so; [ $k = 0 ] && L=$R/speech-enhancement_amd/sehip/libsehip.so
  echo "probe $k" >> $O/stft_probe.log
  SEHIP_LIB=$L timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/stft_probe.log 2>&1 || exit $?
done
