# End-to-end fps vs the smallest tail chunk (same box, interleaved runs).
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for tm in 64 32 16; do
    H2J_TAIL_MIN=$tm timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/t.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/t.json')); s=d['stages_ms_per_step']; print('tail_min $tm', round(d['value'],1), 'fps total', s['total_ms'], 'parse', s['parse_ms'], 'chunks', d['roofline']['frames_per_launch'])"
  done
done
