# model + 16-bit conv tests, then configs 2/3 timing and kernel-trace profiles
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fix4}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  $R/tests/test_gpu_models.py $R/tests/test_gpu_conv_x3.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash $R/tools/gpu_cfg_prof.sh ${1:-fix4}/cfg
