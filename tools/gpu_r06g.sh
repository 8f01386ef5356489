# round-6 batch script (the last one run: final-HEAD evidence, tools/gpu_final.sh parts 1-4 -> profiles/r06fin4/)
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_final.sh r06fin4 1
bash tools/gpu_final.sh r06fin4 2
bash tools/gpu_final.sh r06fin4 3
bash tools/gpu_final.sh r06fin4 4
