# r04fin: the round-4 evidence run: the whole -m gpu suite, smoke(), rocprofv3 kernel stats +
# FETCH_SIZE / WRITE_SIZE passes (profiles/r04fin_*, pmc_k1_<workload>.json) for hevc1080, avc1080
# and hevc2160, then the bench lines (hevc1080 = the driver's default line; avc1080, hevc2160, mixed).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04fin_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r04fin_tests.log | head -30; tail -5 gpurun_out/r04fin_tests.log; exit 1; }
tail -1 gpurun_out/r04fin_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04fin_smoke.log 2>&1 || { tail -5 gpurun_out/r04fin_smoke.log; exit 1; }
tail -1 gpurun_out/r04fin_smoke.log
WLS="hevc1080 avc1080 hevc2160" bash tools/gpu_prof2.sh r04fin
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04fin_hevc1080.json 2> gpurun_out/bench_r04fin_hevc1080.err || { tail -5 gpurun_out/bench_r04fin_hevc1080.err; exit 1; }
for wl in avc1080 hevc2160 mixed; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 --workload $wl --no-aim > gpurun_out/bench_r04fin_$wl.json 2> gpurun_out/bench_r04fin_$wl.err || { tail -5 gpurun_out/bench_r04fin_$wl.err; exit 1; }
done
for f in gpurun_out/bench_r04fin_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d.get('value_aim'), d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d.get('hbm_resident_fps'), d.get('outputs_verified'))" $f; done
