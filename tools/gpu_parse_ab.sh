# Host parse A/B on the GPU box CPU (no GPU use): parse_bench builds given in BINS (tools/parse_bench),
# 1 thread, interleaved, 3 rounds per stream set; prints ms/frame.
cd $GRAFT_REPO_ROOT/tools/parse_bench
for set in ${SETS:-bench bench264 bench_heavy}; do
  for r in 1 2 3; do
    for b in ${BINS:-pb_A pb_B}; do
      echo "$set $b $(./$b ../../tests/golden/$set/*.h26? -r ${REPS:-6} -t 1 | awk '{print $3}')"
    done
  done
done
