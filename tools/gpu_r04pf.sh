# r04pf: same-box A/B: H.264 parser with the inline CABAC engine (build/h264inl, CabacT<true>) vs current
# ("old" below = build/h264inl; the kernels are the same), ABAB.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in new old; do
    for wl in avc1080 mixed; do
      if [ $v = old ]; then export H2J_LIB_DIR=$PWD/h264-h265-to-jpeg_amd/build/h264inl; else unset H2J_LIB_DIR; fi
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --workload $wl --no-aim --no-cpu-baseline --no-single-call > gpurun_out/r04pf_${wl}_${v}_$r.json 2> gpurun_out/r04pf_${wl}_${v}_$r.err || { tail -5 gpurun_out/r04pf_${wl}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d.get('parse_core_us_per_kb'), d['host_cpu_busy_cores'])" gpurun_out/r04pf_${wl}_${v}_$r.json
    done
  done
done
