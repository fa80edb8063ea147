# HIP stream-priority A/B of the train step (bench.py, one box): main step stream and
# CCBAM side stream priorities vs the deferred weight-grad side stream
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prio}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --compare "
timeout -k 10 200 python3 $B "" > $O/a_default.json 2> $O/a.err
SEHIP_MAIN_PRIO=-1 timeout -k 10 200 python3 $B "" > $O/b_main.json 2> $O/b.err
SEHIP_MAIN_PRIO=-1 SEHIP_CCBAM_PRIO=-1 timeout -k 10 200 python3 $B "" > $O/c_main_ccbam.json 2> $O/c.err
timeout -k 10 200 python3 $B "" > $O/d_default2.json 2> $O/d.err
echo ok > $O/ok
