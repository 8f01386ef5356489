# r03j: H.264 deblocking cycle accounting (PROF build, avc1080)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/k1prof.py tests/golden/bench264/avc1080_00.h264 512 2>&1 | tee gpurun_out/r03j_k1prof_avc.log
