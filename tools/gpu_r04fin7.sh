# r04fin7: final state of round 4: GPU suite + smoke + hevc1080 bench line (20 steps).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04fin7_tests.log 2>&1 || { tail -30 gpurun_out/r04fin7_tests.log; exit 1; }
tail -1 gpurun_out/r04fin7_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04fin7_smoke.log 2>&1 || { tail -20 gpurun_out/r04fin7_smoke.log; exit 1; }
tail -1 gpurun_out/r04fin7_smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04fin7_hevc1080.json 2> gpurun_out/bench_r04fin7_hevc1080.err || { tail -5 gpurun_out/bench_r04fin7_hevc1080.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d.get('value_aim'), d.get('parse_core_us_per_kb'), d.get('host_thread_sweep_fps'), d.get('outputs_verified'))" gpurun_out/bench_r04fin7_hevc1080.json
