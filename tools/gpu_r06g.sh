# round-6 batch: GPU suite + same-box A/B against build/base (HEAD before: K4c FDCT on column pairs, v_pk / v_dot2)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_run.sh r06x tests ab:hevc1080:build/base:3 ab:avc1080:build/base:3
for f in gpurun_out/r06x_ab_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['stages_ms_per_step']; print(sys.argv[1], d['config']['workload'], 'jpeg', round(k['jpeg_ms'],3), 'k1', round(d['roofline']['avg_launch_ms'],3), 'hbm_res', round(d['hbm_resident_fps']), 'verified', d['outputs_verified'])" $f; done
