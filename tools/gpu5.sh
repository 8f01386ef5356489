# GPU round trip: full -m gpu suite, then one bench line per workload.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for wl in ${WORKLOADS:-hevc1080 avc1080}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  cat gpurun_out/bench_$wl.json
done
