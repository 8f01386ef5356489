# rocprofv3 kernel-trace stats + two separate PMC passes (FETCH_SIZE / WRITE_SIZE)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
FR=${2:-1024}
WL=${3:-hevc1080}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o stats -- python3 bench.py --workload $WL --steps 2 --warmup 1 --frames $FR --no-cpu-baseline --no-single-call --no-aim > gpurun_out/prof_${TAG}_bench.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o pmc -- python3 bench.py --workload $WL --steps 1 --warmup 0 --frames $FR --no-cpu-baseline --no-single-call --no-aim > gpurun_out/pmc_${TAG}_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${TAG}_write -o pmc -- python3 bench.py --workload $WL --steps 1 --warmup 0 --frames $FR --no-cpu-baseline --no-single-call --no-aim > gpurun_out/pmc_${TAG}_write.log 2>&1
find gpurun_out/prof_$TAG gpurun_out/pmc_${TAG}_fetch gpurun_out/pmc_${TAG}_write -type f | head -20
