# round-6 batch: SAO with 4 CTBs per workgroup (next CTB's loads during this one's filter).  In-tree: 7-wave
# bound; build/v2: 8-wave bound; build/base: HEAD (one CTB per workgroup)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_run.sh r06y tests ab:hevc1080:build/base:3
bash tools/gpu_run.sh r06z ab:hevc1080:build/v2:3
