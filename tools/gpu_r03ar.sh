# r03ar: H.264 deblocking filter with |a - b| as v_sad_u16 and runtime-bound clips as v_med3_i32
# (10 % fewer VALU instructions in h2j_k2_deblock264p): GPU H.264 parity, then same-box A/B
# against the previous build (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_idecoder.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="avc1080" VARIANTS="sad:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
