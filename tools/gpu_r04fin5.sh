# r04fin5: after the HEVC parse engine changes (r04p): the whole -m gpu suite, smoke(), bench lines
# (GPU kernels unchanged since r04fin3, so no new kernel stats / PMC).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04fin5_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r04fin5_tests.log | head -30; tail -5 gpurun_out/r04fin5_tests.log; exit 1; }
tail -1 gpurun_out/r04fin5_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04fin5_smoke.log 2>&1 || { tail -5 gpurun_out/r04fin5_smoke.log; exit 1; }
tail -1 gpurun_out/r04fin5_smoke.log

timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04fin5_hevc1080.json 2> gpurun_out/bench_r04fin5_hevc1080.err || { tail -5 gpurun_out/bench_r04fin5_hevc1080.err; exit 1; }
for wl in avc1080 mixed; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 --workload $wl --no-aim > gpurun_out/bench_r04fin5_$wl.json 2> gpurun_out/bench_r04fin5_$wl.err || { tail -5 gpurun_out/bench_r04fin5_$wl.err; exit 1; }
done
for f in gpurun_out/bench_r04fin5_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d.get('value_aim'), round(d['roofline']['frac'],3), round(d['roofline'].get('avg_launch_ms'),2), round(d.get('hbm_resident_fps')), d.get('parse_core_us_per_kb'), d.get('outputs_verified'))" $f; done
