# A/B of K0 (prep_ms per step) on the reference's own x264 fixture tiled to 1024 pictures: build/base vs current.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in base cur; do
    if [ $v = base ]; then export H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/base; else unset H2J_LIB_DIR; fi
    timeout -k 10 200 python bench.py --workload avc1080 --streams "${STREAMS:-tests/golden/img01.h264}" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/k0_$v.json 2> gpurun_out/k0_$v.err
    python3 -c "import json; d=json.load(open('gpurun_out/k0_$v.json')); s=d['stages_ms_per_step']; print('$v prep', s['prep_ms'], 'ms  recon', s['recon_ms'], 'value', round(d['value'],1))"
  done
done
