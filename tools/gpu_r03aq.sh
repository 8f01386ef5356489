# r03aq: HEVC K1 TBs <= 8x8 read their residual at the TB start (LDS latency off the chain;
# Cb / Cr pairs too): GPU HEVC parity, then same-box A/B against the previous build (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_f3.py tests/test_gpu_idecoder.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -4
WLS="hevc1080 hevc2160" VARIANTS="early:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
