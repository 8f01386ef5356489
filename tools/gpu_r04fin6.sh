# r04fin6: GPU suite + smoke after the last HEVC parse change (scan offset table).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04fin6_tests.log 2>&1 || { tail -30 gpurun_out/r04fin6_tests.log; exit 1; }
tail -2 gpurun_out/r04fin6_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04fin6_smoke.log 2>&1 || { tail -20 gpurun_out/r04fin6_smoke.log; exit 1; }
tail -1 gpurun_out/r04fin6_smoke.log
