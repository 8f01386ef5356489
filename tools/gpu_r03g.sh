# r03g: GPU suite (tiled HEVC residual), kernel stats + FETCH/WRITE for hevc1080, bench line.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_r03g.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03g.log | head -30; tail -30 gpurun_out/pt_r03g.log; exit 1; }
tail -1 gpurun_out/pt_r03g.log
WLS="hevc1080" bash tools/gpu_prof2.sh r03b
timeout -k 10 300 python bench.py --no-cpu-baseline --no-single-call --no-aim --steps 10 --warmup 3 > gpurun_out/b_r03g.json 2> gpurun_out/b_r03g.err || { tail -5 gpurun_out/b_r03g.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_r03g.json')); r=d['roofline']; print('hevc1080', round(d['value'],1), 'fps; hbm_resident', round(d['hbm_resident_fps'],1), 'K1 ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'parse_core', d['parse_core_us_per_kb'])"
