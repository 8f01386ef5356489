# r03k: H.264 deblocking with two MB rows per wave, and K4a's variance sums folded into K3 SAO:
# GPU parity (H.264 + HEVC tests), then A/B against the one-row kernel (H2J_DB264=rows) on
# avc1080 and against the separate K4a pass (H2J_SAO_VAR=0) on hevc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_annexb.py tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -15
WLS=avc1080 VARIANTS="pairs:.: rows:.:H2J_DB264=rows" REPS=2 bash tools/gpu_k1ab.sh
WLS=hevc1080 VARIANTS="fold:.: k4a:.:H2J_SAO_VAR=0" REPS=2 bash tools/gpu_k1ab.sh
