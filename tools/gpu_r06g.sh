# host-only (box CPU): HEVC parser code-generation variants, one thread, min-of-5, 3 interleaved rounds:
# pb_A product flags (clang -march=x86-64-v3 -mtune=znver5), pb_B + -falign-loops=32,
# pb_C + -falign-loops=64, pb_D -march=znver4 (the box's ISA; not portable, for reference)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SETS="bench_aim" BINS="pb_A pb_B pb_C pb_D" ROUNDS=3 REPS=5 timeout -k 10 600 bash tools/gpu_parse_min.sh > gpurun_out/r06w_parse.log 2>&1
cat gpurun_out/r06w_parse.log
