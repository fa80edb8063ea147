# Selected GPU tests, then (if they pass) tools/gpu_evidence.sh:
#   gpurun --timeout 1200 -- bash tools/gpu_tests_then_evidence.sh <tag> <round> <test paths...>
R=$GRAFT_REPO_ROOT; TAG=$1; RND=$2; shift 2
bash $R/tools/gpu_tests.sh $TAG "$@" || exit $?
bash $R/tools/gpu_evidence.sh ${TAG}_ev $RND
