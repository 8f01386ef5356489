# r03: GPU suite, then K1 cycle accounting of the pooled kernel (-DH2J_PROF build, pool on).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_r03a.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03a.log | head -30; tail -30 gpurun_out/pt_r03a.log; exit 1; }
tail -2 gpurun_out/pt_r03a.log
H2J_K1_POOL=4 K1PROF_ASYNC=1 timeout -k 10 120 python3 -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 1024 > gpurun_out/k1prof_pool.log 2>&1 || { echo "k1prof rc=$?"; cat gpurun_out/k1prof_pool.log; exit 1; }
cat gpurun_out/k1prof_pool.log
