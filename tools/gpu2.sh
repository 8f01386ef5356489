set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/probe.py tests/golden/img01.h265 64 3 > gpurun_out/probe.log 2>&1
cat gpurun_out/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof -- python3 tools/probe.py tests/golden/img01.h265 64 2 > gpurun_out/prof1.log 2>&1
find gpurun_out/prof1 -name "*stats*" | head
