# Host CPU use and fps with spinning vs blocking stream waits.
set -e
cd $GRAFT_REPO_ROOT
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
for m in spin block; do
  for wl in ${WLS:-hevc1080}; do
    H2J_SYNC=$m timeout -k 10 200 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sync_${m}_$wl.json 2> gpurun_out/sync_${m}_$wl.err
    python3 -c "import json; d=json.load(open('gpurun_out/sync_${m}_$wl.json')); print('$m $wl', round(d['value'],1), 'cores', d['host_cpu_busy_cores'], {k: round(v,1) for k,v in d['stages_ms_per_step'].items()})"
  done
done
