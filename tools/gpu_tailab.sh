# Same-box comparison of tail-chunk settings (value, tail, K1 frac), hevc1080.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for cfg in "H2J_TAIL_MIN=64" "H2J_TAIL_MIN=128" "H2J_TAIL=0"; do
    env $cfg timeout -k 10 200 python bench.py --workload ${WL:-hevc1080} --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/tab.json 2> gpurun_out/tab.err
    python3 -c "import json; d=json.load(open('gpurun_out/tab.json')); st=d['stages_ms_per_step']; print('$cfg', round(d['value'],1), 'tail', round(st['total_ms']-st['parse_ms'],1), 'K1', round(d['roofline']['avg_launch_ms'],2), 'frac', round(100*d['roofline']['frac'],2))"
  done
done
