# r04f: H.264 K1 cycle accounting (PROF build in build/profavc) on two avc1080 streams, 1024 pictures.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in avc1080_00 avc1080_05 avc1080_07; do
  K1PROF_AVCK1=1 K1PROF_ASYNC=1 H2J_PROF_VARIANT=profavc timeout -k 10 180 python -u tools/k1prof.py tests/golden/bench264/$s.h264 1024 >> gpurun_out/r04f_k1prof_avc.log 2>&1
done
cat gpurun_out/r04f_k1prof_avc.log
