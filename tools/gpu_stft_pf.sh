# ConvSTFT prefetching form A/B (SEHIP_STFT_GPB = frame groups per block; 0 = one group per block)
# + the STFT parity tests with the prefetching form on
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-stftpf}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in ${GPBS:-0 2 3 4 0 2 3 4}; do
  echo "gpb=$v" >> $O/micro.log
  SEHIP_STFT_GPB=$v timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/micro.log 2>&1 || exit $?
done
SEHIP_STFT_GPB=${TEST_GPB:-3} timeout -k 10 300 python3 -u -m pytest -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider $R/tests/test_gpu_stft.py > $O/tests.log 2>&1
echo "pytest rc=$?" >> $O/tests.log
