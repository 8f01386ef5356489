# r03ak: occupancy bounds: HEVC deblocking 8 waves/SIMD (64 VGPRs), K0 7 waves/SIMD (72 VGPRs):
# GPU parity (HEVC + H.264 suites), then same-box A/B against build/base.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="hevc1080 avc1080" VARIANTS="occ:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
