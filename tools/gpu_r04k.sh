# r04k: HEVC K1 pool variants: A (release) = lane laundered per quadrant (2 spilled VGPRs instead of
# 8, none in the quadrant loop); B = A + record loads retired at the DMA waits.  HEVC parity on A and
# B, then same-box A/B/C against HEAD (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04k_tests.log | head -30; tail -5 gpurun_out/r04k_tests.log; exit 1; }
tail -1 gpurun_out/r04k_tests.log
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/varB timeout -k 10 900 python -u -m pytest tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k_testsB.log 2>&1 || { tail -5 gpurun_out/r04k_testsB.log; exit 1; }
tail -1 gpurun_out/r04k_testsB.log
WLS="hevc1080" VARIANTS="base:build/base: A:.: B:build/varB:" REPS=3 bash tools/gpu_k1ab.sh
