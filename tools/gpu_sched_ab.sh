# Gather-kernel scheduling variants (SE_X3_SCHED 1 / 2, libsehip_s1/_s2.so) vs the default:
# conv tests on each, conv_micro forward / data-grad timings, bench steps alternating.
#   gpurun -- bash tools/gpu_sched_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-sched}
O=$R/gpurun_out/$TAG
mkdir -p $O
L=$R/speech-enhancement_amd/sehip
for v in s1 s2; do
  SEHIP_LIB=$L/libsehip_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_join.py > $O/tests_$v.log 2>&1 || { tail -n 30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/tests_$v.log)"
done
for v in base s1 s2 base s1 s2; do
  lib=$L/libsehip.so; [ $v != base ] && lib=$L/libsehip_$v.so
  SEHIP_LIB=$lib timeout -k 10 120 python3 $R/tools/conv_micro.py --layers enc1,enc4,dec5 --passes fwd,data --math f16x3 --iters 10 > $O/micro_$v.log 2>&1 || exit 1
  echo "$v $(grep -hE 'fwd|data' $O/micro_$v.log | tr '\n' ' ')"
done
for v in base s1 s2 base s1 s2; do
  lib=$L/libsehip.so; [ $v != base ] && lib=$L/libsehip_$v.so
  SEHIP_LIB=$lib timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "
import json; d = json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); ob = d['op_breakdown']
print('$v', d['value'], 'utt/s', {x: ob[x]['ms_per_step'] for x in ob if 'conv' in x})"
done
