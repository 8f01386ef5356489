# r03an: K4a 8-bit MB variance sums by v_dot4_u32_u8 (4 samples per instruction for the sum and
# the sum of squares): GPU JPEG parity, then same-box A/B against build/base.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="avc1080" VARIANTS="dot4:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
