# r04l: SAO with the MB variance sums reduced across the wave before the LDS atomics: HEVC parity,
# then same-box A/B against HEAD (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04l_tests.log | head -30; tail -5 gpurun_out/r04l_tests.log; exit 1; }
tail -1 gpurun_out/r04l_tests.log
WLS="hevc1080" VARIANTS="base:build/base: new:.:" REPS=2 bash tools/gpu_k1ab.sh
