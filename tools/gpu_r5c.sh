# round-5 checks: the pipelined gather (bit identity vs gather_x3, conv / join / model parity),
# joined-conv tests (cat order, 16-bit storage), then the GEMM lab
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_tests.sh r5c tests/test_gpu_conv_x3.py tests/test_gpu_join.py tests/test_gpu_cconv.py tests/test_gpu_oob.py tests/test_gpu_models.py tests/test_gpu_variants.py tests/test_gpu_data_weights.py || exit $?
bash $R/tools/gpu_lab.sh lab1
