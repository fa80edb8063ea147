set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-crnact}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/tools/crn_act_diag.py f32 > $O/diag.log 2>&1
echo ok > $O/ok
