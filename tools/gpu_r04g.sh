# r04g: H.264 K1 (I16x16 / chroma paths without reference arrays, group stores deferred to the next
# MB's window step): H.264 parity, cycle accounting, same-box A/B against HEAD (build/base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_h264.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04g_h264.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04g_h264.log | head -30; tail -5 gpurun_out/r04g_h264.log; exit 1; }
tail -1 gpurun_out/r04g_h264.log
K1PROF_AVCK1=1 K1PROF_ASYNC=1 H2J_PROF_VARIANT=profavc timeout -k 10 180 python -u tools/k1prof.py tests/golden/bench264/avc1080_00.h264 1024 > gpurun_out/r04g_k1prof.log 2>&1
cat gpurun_out/r04g_k1prof.log
WLS="avc1080" VARIANTS="base:build/base: new:.:" REPS=2 bash tools/gpu_k1ab.sh
