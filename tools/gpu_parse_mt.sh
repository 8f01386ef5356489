# Host parse scaling on the GPU box CPU (no GPU use): parse_bench at 1/8/16 threads,
# CPU topology of this process's affinity mask.
cd $GRAFT_REPO_ROOT/tools/parse_bench
python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a[:20])"
lscpu | grep -E "Model name|Thread|Core|Socket|NUMA node\(s\)|MHz" | head -8
for t in 1 8 16; do
  echo "hevc t=$t: $(./parse_bench_bin ../../tests/golden/bench/*.h265 -r $((t*4)) -t $t)"
done
echo "avc t=16: $(./parse_bench_bin ../../tests/golden/bench264/*.h264 -r 64 -t 16)"
