# STFT LDS-pad A/B (stft_micro alternating SEHIP_STFT_PAD=0/1) + STFT tests + re-run of selected tests
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fix1}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in 0 1 0 1; do
  SEHIP_STFT_PAD=$v timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/micro.log 2>&1 || exit $?
  echo "pad=$v" >> $O/micro.log
done
timeout -k 10 600 python3 -u -m pytest -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider \
  $R/tests/test_gpu_stft.py $R/tests/test_gpu_cbn.py $R/tests/test_gpu_dynamic_range.py \
  "$R/tests/test_gpu_step.py::test_frcrn_fork_gradient_handoff_bit_identical" > $O/tests.log 2>&1
echo "pytest rc=$?" >> $O/tests.log
