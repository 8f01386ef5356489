# r04pa: HEVC parse A/B on the box's host CPU (no GPU use): pb_A = HEAD, pb_B = residual coding with
# the coeff_abs_level_remaining positions decoded in their own loop (no per-coefficient escape
# branch, signs taken in the output loop) + same-CTB fast path in same_region.
cd $GRAFT_REPO_ROOT
SETS="bench bench_heavy" BINS="pb_A pb_B" REPS=4 bash tools/gpu_parse_ab.sh
