# round-5: 16-bit joined tests, a step-time A/B of the pipelined gather (in-tree library)
# against the round-4 gather_x3 kernels (libsehip_refx3.so), then the GEMM lab
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_tests.sh r5d tests/test_gpu_join.py || exit $?
bash $R/tools/gpu_step_ab.sh r5d_ab refx3 || exit $?
bash $R/tools/gpu_lab.sh lab1
