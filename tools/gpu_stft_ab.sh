# Alternating A/B of the ConvSTFT / iSTFT micro (tools/stft_micro.py) over libraries, in
# the order given ("cur" = the in-tree library, any other name = a variant build
# made with make variant V=name), three rounds, the order rotated each round:
#   gpurun -- bash tools/gpu_stft_ab.sh <tag> cur <variant> [<variant> ...]
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
L=("$@")
n=${#L[@]}
for r in 0 1 2; do
  for ((i = 0; i < n; i++)); do
    V=${L[$(( (i + r) % n ))]}
    LIB=$R/speech-enhancement_amd/sehip/libsehip.so
    [ "$V" != cur ] && LIB=$R/speech-enhancement_amd/sehip/libsehip_$V.so
    echo "== round $((r + 1)) $V" >> $O/ab.log
    SEHIP_LIB=$LIB timeout -k 10 120 python3 $R/tools/stft_micro.py >> $O/ab.log 2>&1 || exit $?
  done
done
python3 - $O/ab.log <<'PY'
import re, sys, statistics as st
rows = {}
cur = None
for line in open(sys.argv[1]):
    m = re.match(r'== round \d+ (\S+)', line)
    if m: cur = m.group(1); continue
    m = re.match(r'(\w+)\s+([\d.]+) us', line)
    if m and cur: rows.setdefault((cur, m.group(1)), []).append(float(m.group(2)))
for (lib, op), v in sorted(rows.items(), key=lambda x: (x[0][1], x[0][0])):
    print(f"{op:9s} {lib:8s} median {st.median(v):6.1f} us  {v}")
PY
