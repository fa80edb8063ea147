R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5base; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/step_times.py 12 > $O/steps.log 2>&1 || exit $?
timeout -k 10 200 python3 $R/tools/conv_micro.py --layers enc1,dec5,dec3 --math f16x3 --iters 10 > $O/micro.log 2>&1 || exit $?
