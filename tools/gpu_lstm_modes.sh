# LSTM recurrence forms (SEHIP_LSTM_LDS = 0 scalar loads, 1 LDS exchange):
# kernel times of tools/lstm_micro.py under rocprofv3 per form.
#   gpurun --timeout 600 -- bash tools/gpu_lstm_modes.sh <tag>
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  SEHIP_LSTM_LDS=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/m$m -o run -- python3 $R/tools/lstm_micro.py > $O/m$m.log 2>&1 || exit $?
  python3 - $O/m$m/run_kernel_stats.csv >> $O/summary.log <<PY
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'lstm' in r['Name']:
        print('mode $m', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
echo ok > $O/ok
SEHIP_LSTM_LDS=1 timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_lstm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_m3.log 2>&1
echo "pytest rc=$?" >> $O/tests_m3.log
