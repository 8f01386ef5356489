# r03z: final round-3 profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes for
# hevc1080, avc1080 and hevc2160 (summaries and pmc_k1_<workload>.json under profiles/, copied to
# gpurun_out/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WLS="hevc1080 avc1080 hevc2160" bash tools/gpu_prof2.sh r03z
