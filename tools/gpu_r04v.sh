# r04v: mixed batches (configs[4]): the merged K1 launch (h2j_k1_recon_any, 132 spilled VGPRs) vs
# per-kind launches on two streams (build/varS).  Parity of varS on the mixed tests, then A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/varS timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mixed or async or batch" > gpurun_out/r04v_tests.log 2>&1 || { tail -8 gpurun_out/r04v_tests.log; exit 1; }
tail -1 gpurun_out/r04v_tests.log
for rep in 1 2; do
for v in base:. split:build/varS; do
  IFS=: read -r label dir <<< "$v"
  H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/$dir timeout -k 10 400 python bench.py --workload mixed --steps 4 --warmup 1 --no-cpu-baseline --no-single-call --no-aim > gpurun_out/r04v_${label}_$rep.json 2> gpurun_out/r04v_${label}_$rep.err || { tail -5 gpurun_out/r04v_${label}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['avg_launch_ms'], d.get('hbm_resident_fps'), d['stages_ms_per_step'].get('recon_ms'))" gpurun_out/r04v_${label}_$rep.json $label
done
done
