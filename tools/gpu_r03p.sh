# r03p: HEVC deblocking fused into SAO (h2j_k3_dbsao): GPU parity (HEVC, f3, annexb, IDecoder),
# then A/B against K2 + h2j_k3_sao (H2J_DBSAO=0) on hevc1080 and hevc2160.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_f3.py tests/test_gpu_annexb.py tests/test_gpu_idecoder.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -15
WLS="hevc1080 hevc2160" VARIANTS="fused:.: k2sao:.:H2J_DBSAO=0" REPS=2 bash tools/gpu_k1ab.sh
