# r03v: H.264 deblocking occupancy: 4-wave workgroups (2 row pairs per wave-round... ) bounded to
# 3 waves per SIMD with global line buffers (3 workgroups per CU, 12 waves, against one 8-wave
# workgroup at 208 VGPRs): GPU H.264 parity, then same-box A/B against build/base on avc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_f3.py tests/test_gpu_annexb.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="avc1080" VARIANTS="occ:.: base:build/base:" REPS=2 bash tools/gpu_k1ab.sh
