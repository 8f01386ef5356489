# Same-box A/B of end-to-end bench lines: build/base (previous commit) vs the current build,
# alternating twice per workload.
set -e
cd $GRAFT_REPO_ROOT
for wl in ${WLS:-hevc1080}; do
  for r in 1 2; do
    for v in base cur; do
      if [ $v = base ]; then export H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/base; else unset H2J_LIB_DIR; fi
      timeout -k 10 200 python bench.py --workload $wl --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
      python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); st=d['stages_ms_per_step']; print('$wl $v', round(d['value'],1), 'parse', round(st['parse_ms'],1), 'total', round(st['total_ms'],1), 'tail', round(st['total_ms']-st['parse_ms'],1))"
    done
  done
done
