# Quick GPU check: full -m gpu suite, then one short bench line per workload (no CPU baseline).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for wl in ${WLS:-hevc1080 avc1080}; do
  timeout -k 10 200 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_$wl.json 2> gpurun_out/q_$wl.err
  python -c "import json; d=json.load(open('gpurun_out/q_$wl.json')); print('$wl', round(d['value'],1), 'fps gpu', round(d['gpu_pipeline_fps'],1), 'K1', round(d['roofline']['avg_launch_ms'],3), 'ms', {k: round(v,1) for k,v in d['stages_ms_per_step'].items()})"
done
