# Host parse speed on the GPU box CPU (no GPU use): old vs new parse_bench binaries.
cd $GRAFT_REPO_ROOT/tools/parse_bench
for b in ${BINS:-parse_bench_old parse_bench_bin}; do
  for set in "../../tests/golden/bench/*.h265" "../../tests/golden/bench264/*.h264"; do
    echo "$b $set: $(./$b $set -r 6 -t 1)"
  done
done
