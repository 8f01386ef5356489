# Per-kernel time split (rocprofv3 kernel trace) for one workload.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
WL=${1:-avc1080}
TAG=${2:-kstats}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$WL -o stats -- python3 bench.py --workload $WL --steps 1 --warmup 1 --no-cpu-baseline --no-aim > gpurun_out/${TAG}_${WL}.log 2>&1
f=$(find gpurun_out/${TAG}_$WL -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows: print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), ('%.2f' % (float(r['TotalDurationNs'])/1e6)).rjust(10), 'ms total', ('%.3f' % (float(r['AverageNs'])/1e6)).rjust(9), 'ms avg')
"
