# ConviSTFT in-place kernel: frame pairs per block A/B + STFT parity tests per variant
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-istftab}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for p in ${PAIRS:-4 8}; do
  SEHIP_ISTFT_IP_PAIRS=$p timeout -k 10 120 python3 -u -m pytest $R/tests/test_gpu_stft.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_p$p.log 2>&1
  echo "istft pairs $p" >> $O/micro.log
  SEHIP_ISTFT_IP_PAIRS=$p timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/micro.log 2>&1
done
echo ok > $O/ok
