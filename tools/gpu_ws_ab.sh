# Warp-specialised split-fp16 gather GEMM (csrc/cconv_ws.hpp, SEHIP_X3_WS=1..4 = variant
# 0..3) against gather_x3_kernel (SEHIP_X3_WS unset): optional parity tests with a variant
# on, conv_micro data-grad timings of every variant, SQ counters of the default and one
# variant, optional bench steps.
#   gpurun -- bash tools/gpu_ws_ab.sh <tag> [tests: variant|0] [sq: variant|0] [bench: variant|0]
R=$GRAFT_REPO_ROOT
TAG=${1:-ws}
TESTS=${2:-0}
SQ=${3:-0}
BENCH=${4:-0}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "$TESTS" != 0 ]; then
  SEHIP_X3_WS=$TESTS timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_join.py > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
  tail -n 1 $O/tests.log
fi
for ws in ${WSV:-0 1 2 3 4}; do
  SEHIP_X3_WS=$ws timeout -k 10 120 python3 $R/tools/conv_micro.py --layers dec5,dec3 --passes data --math f16x3 --iters 10 > $O/micro_ws$ws.log 2>&1 || exit 1
  echo "ws=$ws $(grep -h data $O/micro_ws$ws.log | tr '\n' ' ')"
done
if [ "$SQ" != 0 ]; then
  cd /tmp && export TMPDIR=/tmp
  for ws in 0 $SQ; do
    SEHIP_X3_WS=$ws timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq_ws$ws --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 --iters 2 > $O/sq_ws$ws.log 2>&1 || exit 1
  done
  cd $R
fi
if [ "$BENCH" != 0 ]; then
  for ws in 0 $BENCH; do
    SEHIP_X3_WS=$ws timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/bench_ws$ws.json 2> $O/bench_ws$ws.err || exit 1
    python3 -c "
import json; d = json.loads(open('$O/bench_ws$ws.json').read().strip().splitlines()[-1])
print('ws=$ws', d['value'], 'utt/s', d['op_breakdown']['conv_data_joined_f16x3'])"
  done
fi
