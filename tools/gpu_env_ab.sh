# same-box A/B of an environment knob on the default bench: bash tools/gpu_env_ab.sh <tag> VAR v0 v1
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in $3 $4; do
    env $2=$v timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --compare "" > $O/${2}_${v}_$rep.json 2> $O/${2}_${v}_$rep.err
  done
done
echo ok > $O/ok
