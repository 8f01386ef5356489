# r04z: HEVC K1 with a full-availability fast path (no substitution search when every reference
# is available): HEVC parity, same-box A/B against HEAD (build/base) on hevc1080 and hevc2160.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_tests.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04z_tests.log | head -30; tail -5 gpurun_out/r04z_tests.log; exit 1; }
tail -1 gpurun_out/r04z_tests.log
WLS="hevc1080 hevc2160" VARIANTS="base:build/base: new:.:" REPS=2 bash tools/gpu_k1ab.sh
