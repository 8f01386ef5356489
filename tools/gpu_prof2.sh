# rocprofv3 kernel stats + FETCH/WRITE PMC passes for workloads, then the summaries.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
for wl in ${WLS:-hevc1080 avc1080}; do
  bash tools/gpu_prof.sh ${TAG}_$wl 1024 $wl > /dev/null
  python3 tools/prof_summary.py ${TAG}_$wl $wl > /dev/null
  cp profiles/${TAG}_${wl}_summary.md gpurun_out/ 2>/dev/null || true
  cp profiles/${TAG}_${wl}_kernel_stats.csv gpurun_out/ 2>/dev/null || true
  cp profiles/pmc_k1_${wl}.json gpurun_out/pmc_k1_${wl}.json 2>/dev/null || true
  head -14 profiles/${TAG}_${wl}_summary.md
done
