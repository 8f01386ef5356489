# round-6 batch: GPU suite, end-to-end A/B of the host library (clang -mtune=znver5 parsers) against build/gcchost,
# H.264 parse flags on the box CPU
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06i tests ab:hevc1080:build/gcchost:4 ab:avc1080:build/gcchost:4
SETS="bench264 bench264_heavy bench_aim" BINS="pb_A pb_B" ROUNDS=3 REPS=5 timeout -k 10 500 bash tools/gpu_parse_min.sh > gpurun_out/r06i_parse.log 2>&1
cat gpurun_out/r06i_parse.log
