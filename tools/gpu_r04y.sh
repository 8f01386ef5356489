# r04y: H.264 K1 luma + chroma staged in 8-MB groups at 8 bits (128 / 64-byte rows): H.264 parity, K1 HBM PMC,
# same-box A/B against HEAD (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y_tests.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04y_tests.log | head -30; tail -5 gpurun_out/r04y_tests.log; exit 1; }
tail -1 gpurun_out/r04y_tests.log
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_h264 avc1080 > gpurun_out/r04y_pmc_k1.txt 2>&1
cat gpurun_out/r04y_pmc_k1.txt
WLS="avc1080" VARIANTS="base:build/base: new:.:" REPS=2 bash tools/gpu_k1ab.sh
