# r04h: K1 waits (H.264: no spills, register loads retired at DMA waits; HEVC: record batches and
# next-CTB records retired at DMA waits): H.264 + HEVC parity, H.264 cycle accounting, same-box
# A/B against HEAD (build/base) on avc1080 and hevc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_hevc.py tests/test_gpu_benchsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/r04h_tests.log | head -30; tail -5 gpurun_out/r04h_tests.log; exit 1; }
tail -1 gpurun_out/r04h_tests.log
K1PROF_AVCK1=1 K1PROF_ASYNC=1 H2J_PROF_VARIANT=profavc timeout -k 10 180 python -u tools/k1prof.py tests/golden/bench264/avc1080_00.h264 1024 > gpurun_out/r04h_k1prof.log 2>&1
cat gpurun_out/r04h_k1prof.log
WLS="avc1080 hevc1080" VARIANTS="base:build/base: new:.:" REPS=2 bash tools/gpu_k1ab.sh
