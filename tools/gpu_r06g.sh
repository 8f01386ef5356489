# round-6 batch: plane diff, GPU suite + same-box A/B against build/base (HEAD before: K0 closed-form
# masks, row-wise map stores, batched 4x4 transform skip)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/diag/k0_diff.py r06n3 tests/golden/img01.h265 tests/golden/bench_aim/hevc1080a_00.h265 tests/golden/hevc/p01*.h265 tests/golden/hevc/p05*.h265
bash tools/gpu_run.sh r06n tests ab:hevc1080:build/base:3
for f in gpurun_out/r06n_ab_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], 'prep', round(d['stages_ms_per_step']['prep_ms'],3), 'k1', round(d['roofline']['avg_launch_ms'],3), 'verified', d['outputs_verified'])" $f; done
