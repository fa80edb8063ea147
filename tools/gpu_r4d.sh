# conv / STFT / model / CL16 tests, the STFT micro, three default bench runs and an A/B of
# the CL16 copies, then config 2 with its kernel stats:
#   gpurun --timeout 1200 -- bash tools/gpu_r4d.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_stft.py $R/tests/test_gpu_models.py $R/tests/test_gpu_cl16.py -x -v -s -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python3 $R/tools/stft_micro.py > $O/stft.log 2>&1 || exit $?
bash $R/tools/gpu_ab.sh ${TAG}_ab "" "SEHIP_CL16=1" "" "SEHIP_CL16=1" || exit $?
timeout -k 10 200 python3 $R/tools/bench_configs.py --configs 2 --storage bf16 --iters 10 > $O/cfg2.jsonl 2>> $O/cfg.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 $R/tools/bench_configs.py --configs 2 --storage bf16 --iters 5 > $O/prof2.log 2>&1 || exit $?
echo ok > $O/ok
