# Variant libraries (make variant V=name) against the default one on the f16x3
# gather GEMM: bit-identity of the dec5 data-grad (tools/bm_check.py) and the
# conv micro timing of the given layers / passes.
#   gpurun --timeout 600 -- bash tools/gpu_lib_micro.sh <tag> <layers> <passes> <variants...>
R=$GRAFT_REPO_ROOT
TAG=${1:-libmicro}; LAYERS=${2:-dec5}; PASSES=${3:-data}; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/bm_check.py $O/def.pt > $O/check.log 2>&1 || exit $?
timeout -k 10 200 python3 $R/tools/conv_micro.py --layers $LAYERS --passes $PASSES --math f16x3 > $O/micro_def.log 2>&1 || exit $?
for v in "$@"; do
  L=$R/speech-enhancement_amd/sehip/libsehip_$v.so
  SEHIP_LIB=$L timeout -k 10 120 python3 $R/tools/bm_check.py $O/$v.pt >> $O/check.log 2>&1 || exit $?
  python3 -c "import torch; a=torch.load('$O/def.pt'); b=torch.load('$O/$v.pt'); print('$v', {k: (bool(torch.equal(a[k], b[k])), float((a[k]-b[k]).abs().max())) for k in a})" >> $O/check.log 2>&1
  SEHIP_LIB=$L timeout -k 10 200 python3 $R/tools/conv_micro.py --layers $LAYERS --passes $PASSES --math f16x3 > $O/micro_$v.log 2>&1 || exit $?
done
rm -f $O/*.pt
