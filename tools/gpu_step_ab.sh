# Alternating per-step A/B of the FRCRN bench step (tools/step_times.py, median of the
# steps after the third) between the in-tree library and variant builds, three rounds,
# so a box that slows down under load affects every library alike:
#   gpurun -- bash tools/gpu_step_ab.sh <tag> <variant> [<variant> ...]
# (a variant "env:NAME=value" runs the in-tree library with that environment setting)
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
med() { python3 -c "import re,sys,statistics as s; v=[float(m.group(1)) for m in re.finditer(r'step +\d+ +([\d.]+) ms', open(sys.argv[1]).read())][3:]; print(f'{s.median(v):7.2f} ms median of {len(v)}  min {min(v):7.2f}')" $1; }
for r in 1 2 3; do
  timeout -k 10 200 python3 $R/tools/step_times.py 10 > $O/cur_$r.log 2>&1 || exit $?
  echo "round $r cur  $(med $O/cur_$r.log)" | tee -a $O/ab.log
  for V in "$@"; do
    case $V in
      env:*) E=${V#env:}; F=$(echo $E | tr '=' '_') ;;
      *) E=SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so; F=$V ;;
    esac
    env $E timeout -k 10 200 python3 $R/tools/step_times.py 10 > $O/${F}_$r.log 2>&1 || exit $?
    echo "round $r $V  $(med $O/${F}_$r.log)" | tee -a $O/ab.log
  done
done
