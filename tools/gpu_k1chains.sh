# K1 timing experiments: both chains, chroma chain only (exp3), luma chain only (exp4); 1 and 256 pictures.
set -e
cd $GRAFT_REPO_ROOT
S=${1:-tests/golden/bench/hevc1080_00.h265}
for v in prof exp3 exp4; do
  for n in 1 256; do
    echo "== $v n=$n"
    H2J_PROF_VARIANT=$v timeout -k 10 120 python3 tools/k1prof.py $S $n | head -1
  done
done
