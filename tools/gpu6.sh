# GPU round trip: -m gpu suite, then bench lines for chunk sizes / workloads.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-hevc1080:1024 hevc1080:256 hevc1080:128 avc1080:1024 avc1080:256}; do
  wl=${cfg%%:*}; ch=${cfg##*:}
  H2J_CHUNK=$ch timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${wl}_c$ch.json 2> gpurun_out/bench_${wl}_c$ch.err
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${wl}_c$ch.json')); print('$wl chunk $ch', round(d['value'],1), 'fps', {k: round(v,1) for k,v in d['stages_ms_per_step'].items()})"
done
