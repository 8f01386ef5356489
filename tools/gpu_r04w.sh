# r04w: HEVC K1 pool cycle accounting (PROF build) and SQ counters on hevc1080.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K1PROF_ASYNC=1 H2J_PROF_VARIANT=prof timeout -k 10 180 python -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 1024 > gpurun_out/r04w_k1prof.log 2>&1
cat gpurun_out/r04w_k1prof.log
bash tools/gpu_pmc_kernel.sh h2j_k1_recon_hevc_pool hevc1080 > gpurun_out/r04w_pmc_sq.txt 2>&1
cat gpurun_out/r04w_pmc_sq.txt
