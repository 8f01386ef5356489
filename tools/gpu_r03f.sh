# r03f: host parse A/B of the CABAC steps; kernel stats + FETCH/WRITE passes for hevc1080 and
# avc1080 (profiles/r03a_*, pmc_k1_*.json); GPU suite.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BINS="pb_C3 pb_G pb_H pb_J" SETS="bench bench264 bench_heavy" ROUNDS=5 REPS=5 bash tools/gpu_parse_min.sh
WLS="hevc1080 avc1080" bash tools/gpu_prof2.sh r03a
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_r03f.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03f.log | head -30; tail -30 gpurun_out/pt_r03f.log; exit 1; }
tail -1 gpurun_out/pt_r03f.log
