# Final-HEAD evidence for one round: GPU suite + smoke + the driver's default bench line (part 1), bench lines of
# the four workloads (part 2), rocprof kernel stats + FETCH / WRITE PMC summaries of the four workloads (part 3).
#   gpurun -- bash tools/gpu_final.sh TAG 1|2|3
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
case $2 in
1)
  bash tools/gpu_run.sh $TAG tests smoke
  cp gpurun_out/${TAG}_tests.log gpurun_out/${TAG}_gpu_tests.txt
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err
  tail -c 600 gpurun_out/${TAG}_bench_default.json ;;
2)
  bash tools/gpu_run.sh $TAG bench:hevc1080:20 bench:avc1080:20 bench:hevc2160:10 bench:mixed:10 ;;
ab)  # an environment A/B before the final lines: ab VAR "V1 V2" WL
  bash tools/gpu_ab_env.sh $TAG $3 "$4" $5 3 ;;
3)
  bash tools/gpu_run.sh $TAG prof:hevc1080 prof:avc1080 ;;
4)
  bash tools/gpu_run.sh $TAG prof:hevc2160 prof:mixed ;;
esac
