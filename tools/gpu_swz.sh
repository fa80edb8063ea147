# Conflict-free LDS swizzles (variant build V=swz, -DSEHIP_SWZ2=1): FRCRN gradients bit-identical
# to the in-tree library, the conv / join / wgrad tests on the variant, LDS bank-conflict PMC of
# the variant, then a same-box bench A/B. gpurun --timeout 1200 -- bash tools/gpu_swz.sh <tag>
R=$GRAFT_REPO_ROOT; T=${1:-swz}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
VLIB=$R/speech-enhancement_amd/sehip/libsehip_swz.so
SEHIP_LIB=$VLIB timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_var.pt || exit $?
timeout -k 10 120 python3 $R/tools/grads_dump.py dump /tmp/g_cur.pt || exit $?
python3 $R/tools/grads_dump.py cmp /tmp/g_var.pt /tmp/g_cur.pt > $O/cmp.log 2>&1
SEHIP_LIB=$VLIB timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_conv_x3.py $R/tests/test_gpu_join.py $R/tests/test_gpu_cconv.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
SEHIP_LIB=$VLIB timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/lds --output-format csv -- python3 $R/tools/conv_micro.py --layers dec5,enc1 --passes fwd,data,weight --math f16x3 --iters 1 > $O/lds.log 2>&1 || exit $?
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-compare"
for i in 1 2; do
  SEHIP_LIB=$VLIB timeout -k 10 200 python3 $B > $O/bench_swz$i.json 2> $O/bench_swz$i.err || exit $?
  timeout -k 10 200 python3 $B > $O/bench_cur$i.json 2> $O/bench_cur$i.err || exit $?
done
echo ok > $O/ok
