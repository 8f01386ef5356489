# round-6 final-HEAD evidence (after the K0 / SAO changes): parts 1-4 of tools/gpu_final.sh in one call
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_final.sh r06fin2 1
bash tools/gpu_final.sh r06fin2 2
bash tools/gpu_final.sh r06fin2 3
bash tools/gpu_final.sh r06fin2 4
