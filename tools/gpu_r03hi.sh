# r03h + r03i in one call
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_r03i.sh
bash tools/gpu_r03h.sh
