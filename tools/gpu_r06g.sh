# round-6: host parse variants on the box CPU (tools/parse_bench pb_A / pb_B / pb_C, see profiles/r06_parse_flags.txt)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SETS="bench_aim bench264" BINS="pb_A pb_B pb_C" ROUNDS=3 REPS=5 timeout -k 10 600 bash tools/gpu_parse_min.sh > gpurun_out/r06j_parse.log 2>&1
cat gpurun_out/r06j_parse.log
