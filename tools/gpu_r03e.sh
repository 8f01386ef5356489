# r03e: host parse A/B (C3 / E / F); K1 HBM bytes with and without the staged row stores; the
# prof build without staging; one full default bench line (aim, thread sweep, CPU baseline).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BINS="pb_C3 pb_E pb_F" SETS="bench bench264" ROUNDS=5 REPS=5 bash tools/gpu_parse_min.sh
echo "== K1 PMC, staged"; MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_hevc hevc1080
echo "== K1 PMC, not staged"; H2J_K1_STAGE=0 MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_hevc hevc1080
H2J_K1_STAGE=0 K1PROF_ASYNC=1 timeout -k 10 90 python3 -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 1024 > gpurun_out/k1prof_nostage.log 2>&1 || { echo "k1prof rc=$?"; cat gpurun_out/k1prof_nostage.log; exit 1; }
cat gpurun_out/k1prof_nostage.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03e.json 2> gpurun_out/bench_r03e.err || { tail -5 gpurun_out/bench_r03e.err; exit 1; }
cat gpurun_out/bench_r03e.json
