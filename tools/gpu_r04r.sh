# r04r: H.264 parse speed on the box's host CPU: f76aaa6 (before MBAFF / PAFF) vs HEAD (neighbour
# derivation inline again for frames), both with ROCm clang as the product builds it.
cd $GRAFT_REPO_ROOT
SETS="bench264" BINS="pb_old pb_mbaff pb_new" REPS=4 bash tools/gpu_parse_ab.sh
