# host-only (box CPU): two pictures' HEVC parsers on one thread, switched before every residual
# block (pb_coro) or every coefficient sub-block (pb_coro_sb), against the sequential parse
# (tools/parse_bench/coro.h)
set -e
cd "$GRAFT_REPO_ROOT/tools/parse_bench"
mkdir -p ../../gpurun_out
for b in pb_coro pb_coro_sb; do
  echo "== $b"
  timeout -k 10 300 ./$b ../../tests/golden/bench_aim/*.h265 -r 1 -c
done 2>&1 | tee ../../gpurun_out/r06o_coro.log
