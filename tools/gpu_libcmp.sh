# Bit-identity of the FRCRN train-step gradients between a variant library
# (make variant V=name) and the in-tree one, then a same-box A/B of the
# default bench step against the variant:
#   gpurun --timeout 1200 -- bash tools/gpu_libcmp.sh <tag> <variant>
R=$GRAFT_REPO_ROOT
TAG=$1; V=$2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
VLIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so
SEHIP_LIB=$VLIB timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_var.pt || exit $?
timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_cur.pt || exit $?
python3 $R/tools/grads_dump.py cmp /tmp/g_var.pt /tmp/g_cur.pt > $O/cmp.log 2>&1
cat $O/cmp.log
bash $R/tools/gpu_ab.sh $TAG "SEHIP_LIB=$VLIB"
