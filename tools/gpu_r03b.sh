# r03b: GPU suite (release build), a short bench line, then the -DH2J_PROF pool kernel at P = 1, 2, 4
# (256 / 512 / 1024 pictures), each bounded, stopping at the first failure.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_r03b.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03b.log | head -30; tail -30 gpurun_out/pt_r03b.log; exit 1; }
tail -1 gpurun_out/pt_r03b.log
timeout -k 10 200 python bench.py --workload hevc1080 --steps 6 --warmup 2 --no-cpu-baseline --no-single-call --no-aim > gpurun_out/b_r03b.json 2> gpurun_out/b_r03b.err || { tail -5 gpurun_out/b_r03b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_r03b.json')); r=d['roofline']; print('hevc1080', round(d['value'],1), 'fps; hbm_resident', round(d['hbm_resident_fps'],1), 'K1 ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'parse_core_us_per_kb', d['parse_core_us_per_kb'], {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})"
for n in 256 512 1024; do
  K1PROF_ASYNC=1 timeout -k 10 60 python3 -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 $n > gpurun_out/k1prof_$n.log 2>&1 || { echo "k1prof $n rc=$?"; cat gpurun_out/k1prof_$n.log; exit 1; }
  cat gpurun_out/k1prof_$n.log
done
