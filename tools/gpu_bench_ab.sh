# Same-box A/B of the end-to-end bench line (host + GPU) for two library builds:
#   B_DIR=<dir of the B build> WL=hevc1080 bash tools/gpu_bench_ab.sh
cd $GRAFT_REPO_ROOT
PKG=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd
for rep in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then D=$PKG; else D=$PKG/${B_DIR:-build/base}; fi
    H2J_LIB_DIR=$D timeout -k 10 200 python bench.py --workload ${WL:-hevc1080} --steps ${STEPS:-6} --no-cpu-baseline --no-single-call --no-aim > gpurun_out/bab_$v$rep.json 2> gpurun_out/bab_$v$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/bab_$v$rep.json')); print('$v$rep', round(d['value'],1), d['host_cpu_busy_cores'])"
  done
done
