# PMC counters of one kernel (regex $1) on workload $2 (1024 pictures, one step), two passes:
# SQ instruction mix / waits (default) or MODE=hbm: FETCH_SIZE then WRITE_SIZE (KiB).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-h2j_k3_sao}
WL=${2:-hevc1080}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
if [ "${MODE:-sq}" = hbm ]; then P1="FETCH_SIZE"; P2="WRITE_SIZE"; fi  # KiB, separate passes (MI355X guide)
rm -rf gpurun_out/pmck_1 gpurun_out/pmck_2
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmck_$i -o pmc -- python3 bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline --no-single-call --no-aim > gpurun_out/pmck_$i.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/pmck_*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print(f"{k:24s} {acc[k]:16.0f}  (records {n[k]})")
PY
