# K1 per launch with uniform 256-picture chunks (no shrinking tail), HEVC 1080p and 4K.
set -e
cd $GRAFT_REPO_ROOT
for wl in ${WLS:-hevc1080 hevc2160}; do
  H2J_TAIL=0 timeout -k 10 200 python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/k1u_$wl.json 2> gpurun_out/k1u_$wl.err
  python3 -c "import json; d=json.load(open('gpurun_out/k1u_$wl.json')); print('$wl uniform chunks: K1', round(d['roofline']['avg_launch_ms'],3), 'ms frac', round(100*d['roofline']['frac'],2), '%')"
done
