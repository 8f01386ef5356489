# K0 H.264 group checks: the shipped build's full -m gpu suite, the H.264 suites on an
# experiment build (VARIANT, e.g. build/v62 = 62 records per K0 wave), K0 time of both.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log; exit 1; }
echo "shipped: $(tail -1 gpurun_out/pytest_gpu.log)"
V=${VARIANT:-v62}
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/$V timeout -k 10 120 python -m pytest tests/test_gpu_annexb.py tests/test_gpu_h264.py -q -m gpu --timeout 60 --timeout-method thread > gpurun_out/vx_$V.log 2>&1 || true
echo "$V: $(tail -1 gpurun_out/vx_$V.log)"
for s in tests/golden/img01.h264 "tests/golden/bench264/*.h264"; do
  for d in base $V; do
    H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/$d timeout -k 10 200 python bench.py --workload avc1080 --streams "$s" --steps 2 --warmup 1 --no-cpu-baseline --no-single-call > gpurun_out/k0g.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/k0g.json')); print('$d', '$s', 'prep', d['stages_ms_per_step']['prep_ms'])"
  done
done
