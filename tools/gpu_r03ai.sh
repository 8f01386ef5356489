# r03ai: H.264 K1 I8x8: the filtered corner written by the filter loop (one wave barrier less
# per 8x8 block): GPU H.264 parity, then
# same-box A/B against the previous build (build/base) on avc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_f3.py tests/test_gpu_annexb.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="avc1080" VARIANTS="corner:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
