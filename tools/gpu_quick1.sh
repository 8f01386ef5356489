# GPU parity suite + one hevc1080 and one avc1080 bench line (stage times per step).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_q1.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_q1.log | head -30; tail -30 gpurun_out/pt_q1.log; exit 1; }
tail -1 gpurun_out/pt_q1.log
for wl in ${WLS:-hevc1080 avc1080}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --no-cpu-baseline --no-single-call > gpurun_out/q1_$wl.json 2>gpurun_out/q1_$wl.err || { tail -5 gpurun_out/q1_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q1_$wl.json')); r=d['roofline']; print('$wl', round(d['value'],1), 'hbm_fps', round(d['hbm_resident_fps'],1), 'frac', round(r['frac'],4), {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})"
done
