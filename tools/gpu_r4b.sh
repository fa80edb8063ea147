# CL16 tests, then a same-box A/B of the CL16 weight-grad operands (default vs SEHIP_CL16=0,
# alternating), then the configs-2/3 profiles with PMC (gpu_cfg_prof.sh) and the STFT
# micro with its SQ counters (pmc_stft.sh):
#   gpurun --timeout 1200 -- bash tools/gpu_r4b.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_cl16.py $R/tests/test_gpu_ccbam.py -v -s -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash $R/tools/gpu_ab.sh ${TAG}_ab "SEHIP_CL16=0" "" "SEHIP_CL16=0" || exit $?
bash $R/tools/gpu_cfg_prof.sh ${TAG}_cfg || exit $?
bash $R/tools/pmc_stft.sh ${TAG}_stft || exit $?
exit $rc
