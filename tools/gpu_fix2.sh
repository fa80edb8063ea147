# level-spread gradient test + configs 2/3 timing and kernel-trace profiles
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fix2}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider -s \
  "$R/tests/test_gpu_dynamic_range.py::test_frcrn_level_spread_train_step_grads_vs_fp64" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash $R/tools/gpu_cfg_prof.sh ${1:-fix2}/cfg
