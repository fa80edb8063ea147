R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lw1024; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_lstm_wide.py $R/tests/test_gpu_lstm.py "$R/tests/test_gpu_models.py" -v -m gpu --timeout 200 --timeout-method thread -k "wide or lstm or real_conv or models_vs_golden or crn" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python3 $R/tools/lstm_wide_bench.py --hidden 1024 --cases 4x401,16x401,1x2000 > $O/bench1024.log 2>&1
