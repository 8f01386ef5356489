# Host parse speed on the GPU box CPU (no GPU use): parse_bench variants, 1 thread, 3 runs each.
cd $GRAFT_REPO_ROOT/tools/parse_bench
for set in "../../tests/golden/bench/*.h265" "../../tests/golden/bench264/*.h264"; do
  for r in 1 2 3; do
    for b in ${BINS:-parse_bench_old parse_bench_bin}; do
      echo "$b $set: $(./$b $set -r 6 -t 1 -d)"
    done
  done
done
