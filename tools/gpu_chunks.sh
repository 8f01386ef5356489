cd $GRAFT_REPO_ROOT
for cfg in "256 1" "256 0" "342 0" "512 0" "512 1"; do
  set -- $cfg
  for wl in hevc1080 avc1080; do
    H2J_CHUNK=$1 H2J_TAIL=$2 timeout -k 10 120 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/c.json')); r=d['roofline']; print('$wl chunk $1 tail $2:', round(d['value'],1), 'fps K1', round(r['avg_launch_ms'],2), 'ms frac', round(r['frac'],4), 'total', d['stages_ms_per_step']['total_ms'], 'parse', d['stages_ms_per_step']['parse_ms'])"
  done
done
