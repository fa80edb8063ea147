# GEMM probe variants (make variant V=probe1/probe2): dec5 data-grad f16x3 timing per variant.
#   gpurun --timeout 600 -- bash tools/gpu_probe.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-probe}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "" probe1 probe2; do
  L=$R/speech-enhancement_amd/sehip/libsehip${v:+_$v}.so
  echo "== $v" >> $O/probe.log
  SEHIP_GEMM_BM=256 SEHIP_LIB=$L timeout -k 10 120 python3 $R/tools/conv_micro.py --layers dec5,enc1 --passes data --math f16x3 >> $O/probe.log 2>&1 || exit $?
  SEHIP_GEMM_BM=256 SEHIP_LIB=$L timeout -k 10 120 python3 $R/tools/conv_micro.py --layers dec5 --passes data --math f16x3 >> $O/probe.log 2>&1 || exit $?
done
echo done > $O/ok
