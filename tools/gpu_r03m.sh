# r03m: K1 work balance (LPT slot map for the HEVC pool, heaviest-first H.264 K1 / deblocking map):
# GPU parity (HEVC, H.264, f3, annexb, batch tests), then A/B against frame order (H2J_K1_BALANCE=0).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py tests/test_gpu_f3.py tests/test_gpu_annexb.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -5
WLS="hevc1080 avc1080 hevc2160" VARIANTS="bal:.: frame:.:H2J_K1_BALANCE=0" REPS=2 bash tools/gpu_k1ab.sh
