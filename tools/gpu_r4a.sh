# Round-4 check: the full GPU suite and a bench line (gpu_tb.sh), then
# the wave-local ConvSTFT A/B against its variants and a configs-2/3 A/B of the
# one-term staging depth (variant x3h1 = 32-k rounds):
#   gpurun --timeout 1200 -- bash tools/gpu_r4a.sh <tag> <stft variants...>
R=$GRAFT_REPO_ROOT
TAG=$1; shift
bash $R/tools/gpu_tb.sh $TAG tests
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
bash $R/tools/gpu_stft_ab.sh ${TAG}_stft "$@" > /dev/null || exit $?
O=$R/gpurun_out/${TAG}_cfg
mkdir -p $O
for r in 1 2; do
  timeout -k 10 240 python3 $R/tools/bench_configs.py --configs 2,3 --storage bf16 --iters 10 > $O/cur_$r.jsonl 2>> $O/err.log || exit $?
  SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_x3h1.so timeout -k 10 240 python3 $R/tools/bench_configs.py --configs 2,3 --storage bf16 --iters 10 > $O/x3h1_$r.jsonl 2>> $O/err.log || exit $?
done
exit $rc
