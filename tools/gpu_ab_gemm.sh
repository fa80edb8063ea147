set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r1k; mkdir -p $O
for v in "1 0" "1 1" "2 0" "2 1"; do
  set -- $v
  SEHIP_GEMM_NW=$1 SEHIP_KORDER=$2 timeout -k 10 150 python3 $R/tools/conv_micro.py --layers enc1,dec5,dec3 --passes fwd,data --math bf16x3,bf16x6 --iters 5 > $O/micro_nw$1_k$2.log 2>&1
done
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_join.py $R/tests/test_gpu_cconv.py $R/tests/test_gpu_models.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 $R/bench.py --compare "" --no-cpu-baseline > $O/bench_new.json 2>&1
SEHIP_GEMM_NW=1 SEHIP_KORDER=0 timeout -k 10 300 python3 $R/bench.py --compare "" --no-cpu-baseline > $O/bench_old.json 2>&1
echo ok > $O/ok
