# r04a: the whole -m gpu suite (with the bench-sized parity tests), then the default bench line.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
grep -E "benchsize|PASSED|FAILED" gpurun_out/r04a_tests.log | grep benchsize
timeout -k 10 400 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
cat gpurun_out/r04a_bench.json
