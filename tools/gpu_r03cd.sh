# r03c+d: GPU suite; K1 A/B (staging, residual DMA form); H.264 deblocking A/B; the LDS-accumulator
# -DH2J_PROF pool kernel at P = 1, 2, 4; K1 HBM bytes; host parse A/B on the box CPU.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_r03cd.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_r03cd.log | head -30; tail -30 gpurun_out/pt_r03cd.log; exit 1; }
tail -1 gpurun_out/pt_r03cd.log
BINS="pb_A pb_C3 pb_E" SETS="bench bench264 bench_heavy" ROUNDS=5 REPS=5 bash tools/gpu_parse_min.sh
VARIANTS="stage:.: nostage:.:H2J_K1_STAGE=0 dmabranch:build/dmab:" REPS=2 bash tools/gpu_k1ab.sh
for n in 256 512 1024; do
  K1PROF_ASYNC=1 timeout -k 10 90 python3 -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 $n > gpurun_out/k1prof_$n.log 2>&1 || { echo "k1prof $n rc=$?"; cat gpurun_out/k1prof_$n.log; exit 1; }
  cat gpurun_out/k1prof_$n.log
done
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_hevc hevc1080
