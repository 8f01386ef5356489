# r03fin2: end-of-session profiles and bench lines (after the SAO / deblocking / K0 / K4c steps): rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes for
# hevc1080, avc1080 and hevc2160 (summaries and pmc_k1_<workload>.json under profiles/, copied to
# gpurun_out/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WLS="hevc1080 avc1080" bash tools/gpu_prof2.sh r03fin2
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03fin2_hevc1080.json 2> gpurun_out/bench_r03fin2_hevc1080.err || { tail -5 gpurun_out/bench_r03fin2_hevc1080.err; exit 1; }
for wl in avc1080; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --workload $wl --no-aim > gpurun_out/bench_r03fin2_$wl.json 2> gpurun_out/bench_r03fin2_$wl.err || { tail -5 gpurun_out/bench_r03fin2_$wl.err; exit 1; }
done
for f in gpurun_out/bench_r03fin2_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d.get('value_aim'), d['roofline']['frac'], d['roofline']['avg_launch_ms'], d.get('hbm_resident_fps'))" $f; done
