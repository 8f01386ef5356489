# r03z bench: final round-3 lines at HEAD: the default driver-style bench line (configs[1] + value_aim +
# host thread sweep + CPU baseline), then avc1080 / hevc2160 / mixed lines.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03z_hevc1080.json 2> gpurun_out/bench_r03z_hevc1080.err || { tail -5 gpurun_out/bench_r03z_hevc1080.err; exit 1; }
for wl in avc1080 hevc2160 mixed; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --workload $wl --no-aim > gpurun_out/bench_r03z_$wl.json 2> gpurun_out/bench_r03z_$wl.err || { tail -5 gpurun_out/bench_r03z_$wl.err; exit 1; }
done
for f in gpurun_out/bench_r03z_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d.get('value_aim'), d['roofline']['frac'], d.get('hbm_resident_fps'), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)" $f; done
