# r04c: the whole -m gpu suite (lossless / 12-14-bit / interlace-SPS vectors, tiled H.264 residual,
# SAD/med3 deblocking), then HBM PMC passes of H.264 K1 and deblocking on avc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1 || { grep -E "FAILED|Error|error|assert" gpurun_out/r04c_tests.log | head -30; tail -30 gpurun_out/r04c_tests.log; exit 1; }
tail -2 gpurun_out/r04c_tests.log
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_h264 avc1080 > gpurun_out/r04c_pmc_k1h264.txt 2>&1 && cat gpurun_out/r04c_pmc_k1h264.txt
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k2_deblock264p avc1080 > gpurun_out/r04c_pmc_db264.txt 2>&1 && cat gpurun_out/r04c_pmc_db264.txt
