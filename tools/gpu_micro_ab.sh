# conv GEMM micro (tools/conv_micro.py) for the in-tree library and variant libraries, alternating:
#   gpurun -- bash tools/gpu_micro_ab.sh <tag> <variant> [<variant> ...]   (MICRO_ARGS overrides the conv_micro arguments)
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--layers enc1,dec5,dec3 --math f16x3 --iters 10 --passes fwd,data"}
for r in 1 2; do
  timeout -k 10 200 python3 $R/tools/conv_micro.py $ARGS > $O/cur_$r.log 2>&1 || exit $?
  for V in "$@"; do
    SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so timeout -k 10 200 python3 $R/tools/conv_micro.py $ARGS > $O/${V}_$r.log 2>&1 || exit $?
  done
done
for f in $O/*.log; do echo "== $(basename $f)"; grep -v amdgpu.ids $f; done
