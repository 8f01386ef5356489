# configs[4] K1 per kind (tools/mixed_k1_probe.py) under rocprofv3 kernel stats, one subset per run;
# prints the K1 / deblocking / SAO kernels' total time per subset.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp H2J_CHUNK=1024 H2J_TAIL=0
mkdir -p gpurun_out
TAG=${1:-mk1}
for S in ${SUBSETS:-all hevc h264 hevc_small hevc_4k h264_small h264_4k no_h264_4k no_hevc_4k}; do
  D=gpurun_out/${TAG}_$S
  rm -rf $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o stats -- \
    python3 tools/mixed_k1_probe.py $S > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$S" "$(tail -1 $D.log)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if any(k in n for k in ("k1_recon", "deblock", "k3_sao")):
        out.append(f"{n[:44]} x{r['Calls']} {float(r['TotalDurationNs'])/1e6/2:.3f}")
print(sys.argv[2], "| per transcode (ms):", "; ".join(out))
PY
done
