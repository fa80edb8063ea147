# ConvSTFT in-place kernel: frame pairs per block A/B + STFT parity tests per variant
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-stftab}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for p in ${PAIRS:-4 8}; do
  SEHIP_STFT_IP_PAIRS=$p timeout -k 10 120 python3 -u -m pytest $R/tests/test_gpu_stft.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_p$p.log 2>&1
  SEHIP_STFT_IP_PAIRS=$p timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/micro.log 2>&1
done
echo ok > $O/ok
