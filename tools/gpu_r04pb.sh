# r04pb: parse A/B on the box's host CPU (no GPU use), product flags (HEVC g++, H.264 ROCm clang):
# pb_A = HEAD, pb_B = + HEVC escape loop split / same-CTB fast path, pb_C = + every CABAC engine
# method inlined (refill's tail out of line by value) so a local engine never escapes to memory.
cd $GRAFT_REPO_ROOT
SETS="bench bench264 bench_heavy" BINS="pb_A pb_B pb_C" REPS=4 bash tools/gpu_parse_ab.sh
