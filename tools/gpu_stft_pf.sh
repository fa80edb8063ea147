# ConvSTFT A/B: SEHIP_STFT_GPB (prefetching form, frame groups per block) and SEHIP_STFT_TPB
# (threads per block at nfft 640), alternating; then the STFT parity tests with both on
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-stftpf}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in "0 256" "2 256" "3 256" "0 320" "0 256" "2 256" "3 256" "0 320"; do
  set -- $v
  echo "gpb=$1 tpb=$2" >> $O/micro.log
  SEHIP_STFT_GPB=$1 SEHIP_STFT_TPB=$2 timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/micro.log 2>&1 || exit $?
done
for v in "3 256" "0 320"; do
  set -- $v
  SEHIP_STFT_GPB=$1 SEHIP_STFT_TPB=$2 timeout -k 10 300 python3 -u -m pytest -q -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider $R/tests/test_gpu_stft.py >> $O/tests.log 2>&1
  echo "gpb=$1 tpb=$2 pytest rc=$?" >> $O/tests.log
done
