# r03h: H.264 deblocking A/B (per-edge early-out); the two-chain CABAC interleave microbenchmark
# on the box CPU.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do tools/parse_bench/pb_ilb tests/golden/bench/hevc1080_00.h265 tests/golden/bench/hevc1080_04.h265; done
WLS=avc1080 VARIANTS="base:.: dbskip:build/dbskip:" REPS=3 bash tools/gpu_k1ab.sh
