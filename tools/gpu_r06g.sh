# round-6 final HEAD: GPU suite + smoke + the driver's default bench line (bench.py with no flags: 12 timed steps)
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_final.sh r06fin3 1
bash tools/gpu_r06h.sh
