# mixed workload: merged K1 launch vs separate launches
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for m in 1 0; do
  H2J_K1_MERGE=$m timeout -k 10 200 python bench.py --workload mixed --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/merge_$m.json 2> gpurun_out/merge_$m.err
  python3 -c "import json; d=json.load(open('gpurun_out/merge_$m.json')); print('merge=$m', round(d['value'],1), 'K1', round(d['roofline']['avg_launch_ms'],2), {k: round(v,1) for k,v in d['stages_ms_per_step'].items()})"
done
