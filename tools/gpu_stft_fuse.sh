# ConvSTFT fused first pass: tests, then per-call timing A/B (tools/stft_micro.py) and a kernel trace
R=$GRAFT_REPO_ROOT; T=${1:-stf}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_stft.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  SEHIP_STFT_FUSE=0 timeout -k 10 120 python3 $R/tools/stft_micro.py > $O/micro_off$i.log 2>&1 || exit $?
  SEHIP_STFT_FUSE=1 timeout -k 10 120 python3 $R/tools/stft_micro.py > $O/micro_on$i.log 2>&1 || exit $?
done
SEHIP_STFT_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/stft_micro.py > $O/prof.log 2>&1 || exit $?
echo ok > $O/ok
