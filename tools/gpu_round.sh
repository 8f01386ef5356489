# Full measurement round: -m gpu tests, bench lines (with CPU baseline) per
# workload, rocprofv3 kernel stats + separate FETCH/WRITE PMC passes.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01i}
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for wl in ${WLS:-hevc1080 avc1080}; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/bench_${TAG}_$wl.json 2> gpurun_out/bench_${TAG}_$wl.err
  cat gpurun_out/bench_${TAG}_$wl.json
  bash tools/gpu_prof.sh ${TAG}_$wl 1024 $wl > /dev/null
done
echo done
