# STFT A/B + CBN / CCBAM / level-spread tests + a quick bench line
R=$GRAFT_REPO_ROOT; T=${1:-fix5}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
bash $R/tools/gpu_stft_pf.sh $T/stft || exit $?
timeout -k 10 600 python3 -u -m pytest -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider -s \
  $R/tests/test_gpu_cbn.py $R/tests/test_gpu_ccbam.py $R/tests/test_gpu_join.py $R/tests/test_gpu_models.py \
  "$R/tests/test_gpu_dynamic_range.py::test_frcrn_level_spread_train_step_grads_vs_fp64" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --compare "" > $O/bench.json 2> $O/bench.err
