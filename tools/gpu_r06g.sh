# round-6 batch: SQ counters of the H.264 deblocking and K1 on avc1080 (configs[2])
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06q "pmc:h2j_k2_deblock264p:avc1080:sq" "pmc:h2j_k1_recon_h264:avc1080:sq"
