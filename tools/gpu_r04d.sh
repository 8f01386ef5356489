# r04d: H.264 GPU parity incl. the MBAFF vectors (a31-a36), then the whole suite, then avc1080 kernel times.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_h264.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04d_h264.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04d_h264.log | head -40; tail -5 gpurun_out/r04d_h264.log; exit 1; }
tail -2 gpurun_out/r04d_h264.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || { tail -30 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
WLS="avc1080" VARIANTS="mbaff:.:" REPS=1 bash tools/gpu_k1ab.sh
