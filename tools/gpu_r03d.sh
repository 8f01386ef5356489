# r03d: GPU suite; H.264 deblocking A/B (edge-parallel internal edges vs r03c's line-serial form);
# host parse A/B (CABAC variants) on the box CPU.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_r03d.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03d.log | head -30; tail -30 gpurun_out/pt_r03d.log; exit 1; }
tail -1 gpurun_out/pt_r03d.log
WLS=avc1080 VARIANTS="dbnew:.: dbold:build/dbold:" REPS=2 bash tools/gpu_k1ab.sh
BINS="pb_A pb_C3 pb_E" SETS="bench bench264 bench_heavy" ROUNDS=5 REPS=5 bash tools/gpu_parse_min.sh
