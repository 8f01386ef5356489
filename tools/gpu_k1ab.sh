# A/B of K1 per launch (uniform chunks): current build vs build/base
set -e
cd $GRAFT_REPO_ROOT
for v in base cur; do
  for wl in ${WLS:-hevc1080}; do
    if [ $v = base ]; then export H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/base; else unset H2J_LIB_DIR; fi
    H2J_TAIL=0 timeout -k 10 200 python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${v}_$wl.json 2> gpurun_out/ab_${v}_$wl.err
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${v}_$wl.json')); print('$v $wl K1', round(d['roofline']['avg_launch_ms'],3), 'ms')"
  done
done
