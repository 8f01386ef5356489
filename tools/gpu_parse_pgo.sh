# host-only (box CPU): HEVC / H.264 parse, one thread, min-of-5 per stream, 3 interleaved rounds:
# pb_A = the product build (clang, HEVC parser -mtune=znver5), pb_B = g++ with profile feedback
# (-fprofile-use, profile from the bench / bench_aim / bench264 streams), pb_C = g++ without it
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SETS="bench_aim bench264" BINS="pb_A pb_B pb_C" ROUNDS=3 REPS=5 timeout -k 10 600 bash tools/gpu_parse_min.sh > gpurun_out/r06u_parse.log 2>&1
cat gpurun_out/r06u_parse.log
