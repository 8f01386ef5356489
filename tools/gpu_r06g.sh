# round-6 final-HEAD evidence (after the K4c change): parts 1-4 of tools/gpu_final.sh in one call
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_final.sh r06fin4 1
bash tools/gpu_final.sh r06fin4 2
bash tools/gpu_final.sh r06fin4 3
bash tools/gpu_final.sh r06fin4 4
