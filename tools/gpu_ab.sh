# A/B of environment knobs on the default bench step (no CPU baseline, no op timing, no compare legs):
#   gpurun --timeout 900 -- bash tools/gpu_ab.sh <tag> "ENV=a ENV2=b" "ENV=c" ...
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "" "$@"; do
  echo "== [$cfg]" >> $O/ab.log
  env $cfg timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-op-timing --no-compare > $O/ab_$i.json 2>> $O/ab.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/ab_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> $O/ab.log
  i=$((i+1))
done
echo done > $O/ok
