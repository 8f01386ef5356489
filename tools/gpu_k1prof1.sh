# K1 cycle accounting (prof build), one picture and 128 pictures.
set -e
cd $GRAFT_REPO_ROOT
S=${1:-tests/golden/bench/hevc1080_00.h265}
for n in 1 128; do
  H2J_PROF_VARIANT=${V:-prof} timeout -k 10 120 python3 tools/k1prof.py $S $n
done
