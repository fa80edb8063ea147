# Build the STFT measurement probes (CPU side): each is libsehip.so with stft.hip compiled
# with -DSEHIP_STFT_PROBE=k -> sehip/libsehip_stftp<k>.so. Run on the GPU with
#   for k in 0 1 2 3; do SEHIP_LIB=.../libsehip_stftp$k.so python3 tools/stft_micro.py; done
set -e
cd "$(dirname "$0")/../speech-enhancement_amd"
make -j8 >/dev/null
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize"
for k in ${PROBES:-1 2 3}; do
  mkdir -p build_stftp$k
  $CXX -DSEHIP_STFT_PROBE=$k -c csrc/stft.hip -o build_stftp$k/stft.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $(ls build/*.o | grep -v '/stft.o') build_stftp$k/stft.o \
    -o sehip/libsehip_stftp$k.so
done
