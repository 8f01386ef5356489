# r04u: H.264 parse speed on the box's host CPU: f76aaa6 (before MBAFF / PAFF) vs HEAD (neighbour
# derivation inline again for frames), both with ROCm clang as the product builds it.
cd $GRAFT_REPO_ROOT
SETS="bench bench264 bench_heavy" BINS="pb_cur pb_dec" REPS=4 bash tools/gpu_parse_ab.sh
