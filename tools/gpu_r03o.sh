# r03o: K4c row pass with packed adds + v_dot2 (bit-exact JPEG coefficients): GPU JPEG / HEVC /
# H.264 parity, then K4c time on hevc1080 and avc1080 (rocprofv3 kernel stats).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py tests/test_gpu_f3.py tests/test_gpu_idecoder.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="hevc1080 avc1080" VARIANTS="dot2:.:" REPS=2 bash tools/gpu_k1ab.sh
