# K1 instruction-mix PMC passes (one rocprofv3 run per counter group) on a 256-frame batch.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STREAM=${1:-tests/golden/bench/hevc1080_00.h265}
TAG=${2:-k1mix}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${TAG}_a -o pmc -- python3 tools/probe.py $STREAM 256 1 > gpurun_out/${TAG}_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${TAG}_b -o pmc -- python3 tools/probe.py $STREAM 256 1 > gpurun_out/${TAG}_b.log 2>&1
python3 - <<PY
import csv, glob, collections
for part in "ab":
    f = glob.glob("gpurun_out/${TAG}_%s/**/*counter_collection.csv" % part, recursive=True)
    if not f: print("no csv", part); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        if "recon" in k or "prep" in k or "sao" in k or "deblock" in k:
            print(part, k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
