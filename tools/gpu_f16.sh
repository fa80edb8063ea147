# f16x3 bring-up: conv parity tests (every mode vs fp64), then the train step in
# f16x3 beside the previous default. A test failure (rc 1) does not stop the
# script; a crash, abort or timeout does.
#   gpurun --timeout 900 -- bash tools/gpu_f16.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-f16}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_cconv.py $R/tests/test_gpu_join.py \
  -v -s -m gpu --timeout 120 --timeout-method thread > $O/conv_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/conv_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --math f16x3 --compare "fwd=bf16x6,data=bf16x3,weight=bf16x3,fwd_dec=bf16x3,fwd_dec_min_h=158;bf16x6" --steps 10 --warmup 3 > $O/bench_f16.json 2> $O/bench_f16.err || exit $?
echo done > $O/ok
