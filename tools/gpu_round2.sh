# Round measurement: -m gpu suite, then one default bench line (with the CPU baseline and the
# single-call latency) per workload, plus configs[4] at its per-GPU size (8192 pictures).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_$TAG.log | head -30; tail -5 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for wl in ${WLS:-hevc1080 avc1080 hevc2160 mixed hevc1080_heavy}; do
  timeout -k 10 400 python bench.py --workload $wl > gpurun_out/${TAG}_bench_$wl.json 2> gpurun_out/${TAG}_bench_$wl.err || { tail -5 gpurun_out/${TAG}_bench_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$wl.json')); r=d['roofline']; print('$wl', round(d['value'],1), 'hbm', round(d['hbm_resident_fps'],1), 'frac', round(r['frac'],4), 'own', round(r.get('frac_k1_own',0),4), 'pipe', round(r.get('frac_pipeline',0),4), 'cpu', d['cpu_baseline']['value'])"
done
if [ -z "${SKIP8192:-}" ]; then
  timeout -k 10 600 python bench.py --workload mixed --frames 8192 --steps 2 --warmup 1 --no-cpu-baseline --no-single-call > gpurun_out/${TAG}_bench_mixed8192.json 2> gpurun_out/${TAG}_bench_mixed8192.err || { tail -5 gpurun_out/${TAG}_bench_mixed8192.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_mixed8192.json')); print('mixed8192', round(d['value'],1), 'hbm', round(d['hbm_resident_fps'],1), d['ms_per_step'])"
fi
