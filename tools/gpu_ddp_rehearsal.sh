# GPU DDP tests (flat and hook-based) + a 2-rank bench.py rehearsal on the box's one GPU
# (both ranks on cuda:0 over gloo: exercises FlatDataParallel, the barrier and the
# max-over-ranks timing; the driver's N>1 runs use RCCL on separate GPUs)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ddpr}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_ddp.py -v -m gpu --timeout 240 --timeout-method thread > $O/tests.log 2>&1
[ "$2" = "bench" ] || { echo ok > $O/ok; exit 0; }   # pass "bench" for the 2-rank bench rehearsal
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=2 LOCAL_RANK=0 SEHIP_DIST_BACKEND=gloo
RANK=1 timeout -k 10 300 python3 $R/bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 --no-cpu-baseline --compare "" > $O/bench_r1.json 2> $O/bench_r1.err &
P1=$!
RANK=0 timeout -k 10 300 python3 $R/bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 --no-cpu-baseline --compare "" > $O/bench_r0.json 2> $O/bench_r0.err
wait $P1
echo ok > $O/ok
