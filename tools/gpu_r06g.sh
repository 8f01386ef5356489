# round-6 batch: GPU suite + same-box A/B against build/base (HEAD before: HEVC K1 filtered reference neighbours by DPP
# instead of ds_bpermute)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_run.sh r06t tests ab:hevc1080:build/base:3
for f in gpurun_out/r06t_ab_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['stages_ms_per_step']; print(sys.argv[1], 'k1', round(d['roofline']['avg_launch_ms'],3), 'prep', round(k['prep_ms'],3), 'verified', d['outputs_verified'])" $f; done
bash tools/gpu_parse_pgo.sh
