# Same-box A/B of K1 variants by per-kernel average times (rocprofv3 kernel trace of a short
# bench run), alternating the variants REPS times.  VARIANTS: "label:libdir:ENV=VAL,ENV2=VAL ..."
# (libdir relative to h264-h265-to-jpeg_amd, "." = the release build).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PKG=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd
for wl in ${WLS:-hevc1080}; do
  for rep in $(seq ${REPS:-2}); do
    for v in ${VARIANTS:-base:.:}; do
      IFS=: read -r label dir envs <<< "$v"
      out=gpurun_out/k1ab_${wl}_${label}_$rep
      env ${envs//,/ } H2J_LIB_DIR=$PKG/$dir timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o stats -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-single-call --no-aim > $out.log 2>&1 || { echo "$label failed"; tail -5 $out.log; exit 1; }
      f=$(find $out -name "*kernel_stats.csv" | head -1)
      python3 - "$f" "$wl $label$rep" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    n = re.sub(r'^void ', '', n.replace('(anonymous namespace)::', ''))
    return re.sub(r'^.*::', '', n.split('(')[0]).replace('h2j_', '')
print(sys.argv[2], ' '.join('%s=%.3f' % (short(r['Name']), float(r['AverageNs']) / 1e6) for r in rows[:12]))
PY
    done
  done
done
