# r03af: H.264 deblocking skips the luma edge-16 filter when both MBs of the wave use the 8x8
# transform (uniform branch): GPU H.264 parity, then
# same-box A/B against the previous build (build/base) on avc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_f3.py tests/test_gpu_annexb.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="avc1080" VARIANTS="e16:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
