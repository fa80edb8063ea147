# A/B of variant libraries (make variant V=name) on the default bench step.
#   gpurun --timeout 900 -- bash tools/gpu_lib_ab.sh <tag> <variant names...>
R=$GRAFT_REPO_ROOT
TAG=${1:-libab}; shift
args=()
for v in "$@"; do args+=("SEHIP_LIB=$R/speech-enhancement_amd/sehip/libsehip_$v.so"); done
bash $R/tools/gpu_ab.sh $TAG "${args[@]}"
