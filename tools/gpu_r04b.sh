# r04b: the default bench line (outputs_verified), then the H.264 deblocking SAD/med3 A/B
# (tools/r03ar_db264_sad_med3.patch applied in build/sad) on avc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || { tail -20 gpurun_out/r04b_bench.err; exit 1; }
cat gpurun_out/r04b_bench.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_h264.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -2
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/sad timeout -k 10 300 python -u -m pytest tests/test_gpu_h264.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -2
WLS="avc1080" VARIANTS="base:.: sad:build/sad:" REPS=3 bash tools/gpu_k1ab.sh
