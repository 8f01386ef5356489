# r04m: H.264 deblocking cycle accounting (PROF build, build/prof) and HBM PMC (FETCH / WRITE) of
# H.264 K1 and deblocking on avc1080 after the r04 changes.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K1PROF_ASYNC=1 H2J_PROF_VARIANT=prof timeout -k 10 180 python -u tools/k1prof.py tests/golden/bench264/avc1080_00.h264 1024 > gpurun_out/r04m_dbprof.log 2>&1
cat gpurun_out/r04m_dbprof.log
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k1_recon_h264 avc1080 > gpurun_out/r04m_pmc_k1.txt 2>&1
cat gpurun_out/r04m_pmc_k1.txt
MODE=hbm bash tools/gpu_pmc_kernel.sh h2j_k2_deblock264p avc1080 > gpurun_out/r04m_pmc_db.txt 2>&1
cat gpurun_out/r04m_pmc_db.txt
bash tools/gpu_pmc_kernel.sh h2j_k2_deblock264p avc1080 > gpurun_out/r04m_pmc_db_sq.txt 2>&1
cat gpurun_out/r04m_pmc_db_sq.txt
