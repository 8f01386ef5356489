# round-6 batch: GPU suite, K1 A/B against build/base, mixed K1 split A/B, 4K / mixed bench lines, host parse flags
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06h tests ab:hevc1080:build/base:3
bash tools/gpu_ab_env.sh r06h H2J_K1_SPLIT "0 1" mixed 3
bash tools/gpu_run.sh r06h bench:hevc2160:8
SETS="bench_aim bench" BINS="pb_A pb_B pb_C pb_D" ROUNDS=3 REPS=5 timeout -k 10 500 bash tools/gpu_parse_min.sh > gpurun_out/r06h_parse.log 2>&1
cat gpurun_out/r06h_parse.log
