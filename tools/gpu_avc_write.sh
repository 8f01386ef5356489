set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt.log | head -30; tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python bench.py --workload avc1080 --no-cpu-baseline --no-single-call > gpurun_out/avc.json
python -c "import json; d=json.load(open('gpurun_out/avc.json')); r=d['roofline']; print('avc', round(d['value'],1), 'hbm_fps', round(d['hbm_resident_fps'],1), {k: round(v,2) for k,v in d['stages_ms_per_step'].items()}, 'frac', round(r['frac'],4))"
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o pmc -- python3 bench.py --workload avc1080 --steps 1 --warmup 0 --no-cpu-baseline --no-single-call > gpurun_out/pmcw.log 2>&1
python3 - <<PY
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_w/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k] += float(r["Counter_Value"]); n[k] += 1
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:8]:
    print(f"{k:42s} calls {n[k]:4d}  WRITE {v/1024:.1f} MiB total, per frame {v*1024/1024/1e6:.2f} MB")
PY
