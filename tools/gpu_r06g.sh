# round-6 batch: GPU suite + same-box A/B of this build against build/gcchost (K0 coefficient loads batched)
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06l tests ab:hevc1080:build/gcchost:3
for f in gpurun_out/r06l_ab_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], 'prep', round(d['stages_ms_per_step']['prep_ms'],3), 'k1', round(d['roofline']['avg_launch_ms'],3), 'verified', d['outputs_verified'])" $f; done
