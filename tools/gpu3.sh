set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/bench1.log; exit 1; }
tail -2 gpurun_out/bench1.log
