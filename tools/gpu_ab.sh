# A/B of two builds of the libraries on one box: per-kernel average times (rocprofv3 kernel
# trace) of a short bench run, alternating the builds twice.
#   B_DIR=<dir with the B build> WLS="hevc1080 avc1080" bash tools/gpu_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PKG=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd
for wl in ${WLS:-hevc1080}; do
  for rep in 1 2; do
    for v in A B; do
      if [ $v = A ]; then D=$PKG; else D=$PKG/${B_DIR:-build/ab}; fi
      out=gpurun_out/ab_${wl}_${v}_$rep
      H2J_LIB_DIR=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o stats -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-single-call --no-aim > $out.log 2>&1
      f=$(find $out -name "*kernel_stats.csv" | head -1)
      python3 - "$f" "$wl $v$rep" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(sys.argv[2], 'total %.2f ms |' % (tot / 1e6 / max(1, int(rows[0]['Calls']) if rows else 1) * 1),
      ' '.join('%s=%.3f' % (re.sub(r'^.*::', '', r['Name'].split('(', 2)[-2] if '(' in r['Name'] else r['Name']).replace('h2j_', ''), float(r['AverageNs']) / 1e6) for r in rows[:12]))
PY
    done
  done
done
