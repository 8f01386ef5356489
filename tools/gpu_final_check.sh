# Round-end check: -m gpu suite, smoke(), the box's CPU share, and the hevc1080 bench line at
# several host thread counts (THREADS) around the cgroup quota.
[ -n "$NOSUITE" ] || timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1; [ -n "$NOSUITE" ] || tail -1 gpurun_out/pytest_gpu_final.log
[ -n "$NOSUITE" ] || timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
python3 -c "import os; print('cpus', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for t in ${THREADS:-14 16 18 20}; do
  timeout -k 10 200 python bench.py --workload hevc1080 --threads $t --steps 6 --no-cpu-baseline --no-single-call --no-aim > gpurun_out/thr_$t.json 2> gpurun_out/thr_$t.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/thr_$t.json')); print('threads $t', round(d['value'],1), d['host_cpu_busy_cores'])"
done
