# One gpurun call: STFT parity tests, the gradient gate of tools/grad_modes.py for the
# decoder-forward math variants (fwd_dec), and a bench line per variant.
#   gpurun --timeout 1200 -- bash tools/gpu_fwd_dec.sh <tag>
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fwddec}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
D="fwd=bf16x6,data=bf16x3,weight=bf16x3"
timeout -k 10 200 python3 -u -m pytest $R/tests/test_gpu_stft.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/stft_tests.log 2>&1
timeout -k 10 400 python3 -u $R/tools/grad_modes.py "$D" "$D,fwd_dec=bf16x3,fwd_dec_min_h=158" "$D,fwd_dec=bf16x3,fwd_dec_min_h=77" "$D,fwd_dec=bf16x3,fwd_dec_min_h=37" "$D,fwd_dec=bf16x3,fwd_dec_min_h=0" > $O/grad_modes.log 2>&1
for h in 158 77 37; do
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --compare "" --math "$D,fwd_dec=bf16x3,fwd_dec_min_h=$h" > $O/bench_h$h.json 2> $O/bench_h$h.err
done
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --compare "" > $O/bench_default.json 2> $O/bench_default.err
echo ok > $O/ok
