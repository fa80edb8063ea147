# A/B of HIP stream priorities for the FRCRN step (bench.py headline only): the main
# stream, the CCBAM gate stream and the deferred weight-grad stream at priority -1 (high)
# one at a time, interleaved with the default (all 0); rocm-smi clocks / power between runs.
#   gpurun -- bash tools/gpu_prio_ab.sh <tag> [order, default "gates base main wgrad base"]
R=$GRAFT_REPO_ROOT
TAG=${1:-prio}
ORDER=${2:-gates base main wgrad base}
O=$R/gpurun_out/$TAG
mkdir -p $O
B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
n=0
for v in $ORDER; do
  n=$((n + 1))
  timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp --showuse > $O/smi_$n.txt 2>&1
  case $v in
    main) E=SEHIP_PRIO_MAIN=-1 ;;
    gates) E=SEHIP_PRIO_GATES=-1 ;;
    wgrad) E=SEHIP_PRIO_WGRAD=-1 ;;
    iso) E=SEHIP_OVERLAP=0 ;;
    q8) E=GPU_MAX_HW_QUEUES=8 ;;
    q16) E=GPU_MAX_HW_QUEUES=16 ;;
    *) E=SEHIP_PRIO_NONE=0 ;;
  esac
  env $E timeout -k 10 240 $B > $O/${n}_$v.json 2> $O/${n}_$v.err || exit $?
  grep -h "utt/s" $O/${n}_$v.err
done
timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp --showuse > $O/smi_end.txt 2>&1
echo ok > $O/ok
