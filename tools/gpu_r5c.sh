# round-5 checks: joined-conv tests (cat order, 16-bit storage), then the GEMM lab
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_tests.sh r5c tests/test_gpu_join.py tests/test_gpu_variants.py tests/test_gpu_models.py tests/test_gpu_oob.py || exit $?
bash $R/tools/gpu_lab.sh lab1
