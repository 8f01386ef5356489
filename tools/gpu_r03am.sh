# r03am: HEVC K0 at 8 waves/SIMD (64 VGPRs, 12 spilled) against 7 (72 VGPRs):
# GPU parity (HEVC + H.264 suites), then same-box A/B against build/base.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="hevc1080 hevc2160" VARIANTS="k08:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
