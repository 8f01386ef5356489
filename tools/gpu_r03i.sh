# r03i: H.264 deblocking cycle accounting (PROF build, avc1080) and a host parse A/B of the
# emit_tu in-place construction (pb_K before, pb_L after) on the box CPU.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/k1prof.py tests/golden/bench264/avc1080_00.h264 512 2>&1 | tee gpurun_out/r03i_k1prof_avc.log
BINS="pb_K pb_L" ROUNDS=5 REPS=5 SETS="bench bench_heavy" bash tools/gpu_parse_min.sh | tee gpurun_out/r03i_parse.txt
