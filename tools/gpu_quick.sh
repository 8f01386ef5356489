# Quick GPU check: full -m gpu suite, then one short bench line per workload (no CPU baseline).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for wl in ${WLS:-hevc1080 avc1080}; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-single-call --no-aim ${BENCH_ARGS:-} > gpurun_out/q_$wl.json 2> gpurun_out/q_$wl.err
  python -c "import json; d=json.load(open('gpurun_out/q_$wl.json')); r=d['roofline']; print('$wl', round(d['value'],1), 'fps; hbm_resident', round(d['hbm_resident_fps'],1), 'K1 frac', round(r['frac'],4), {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})"
done
