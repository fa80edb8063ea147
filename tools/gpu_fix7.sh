# new parity tests (B = 64 bench batch, 16-bit join) + a kernel-trace profile of the bench
R=$GRAFT_REPO_ROOT; T=${1:-fix7}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -v -m gpu --timeout 450 --timeout-method thread -p no:cacheprovider -s \
  "$R/tests/test_gpu_models.py::test_frcrn_bench_batch_b64_train_forward_vs_oracle" $R/tests/test_gpu_join.py \
  > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing --no-compare > $O/prof_bench.log 2>&1 || exit $?
