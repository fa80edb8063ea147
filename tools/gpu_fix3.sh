# bf16-storage drift tests + CBN/GEMM overlap micro + configs 2/3 timing and kernel-trace profiles
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fix3}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v -m gpu --timeout 250 --timeout-method thread -p no:cacheprovider -s \
  "$R/tests/test_gpu_models.py::test_bf16_configs_within_oracle_bf16_drift" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 180 python3 $R/tools/overlap_micro.py > $O/overlap.log 2>&1 || exit $?
bash $R/tools/gpu_cfg_prof.sh ${1:-fix3}/cfg
