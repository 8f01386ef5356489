# r04e: H.264 GPU parity incl. the PAFF field pairs (a37-a40) and the strict-mode / malformed cases.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_f3.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04e_h264.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04e_h264.log | head -40; tail -5 gpurun_out/r04e_h264.log; exit 1; }
tail -2 gpurun_out/r04e_h264.log
