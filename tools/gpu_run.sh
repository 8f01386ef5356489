# One parametrised runner for the GPU box (replaces the per-experiment tools/gpu_r0*.sh scripts;
# their results stay in profiles/).  Every step runs under its own time limit and the first
# failing step ends the call (set -e), so a fault or hang never starts another GPU step.
#
#   gpurun -- bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP:
#   tests[:EXPR]              -m gpu suite (EXPR: a pytest -k expression)     -> gpurun_out/TAG_tests.log
#   smoke                     __graft_entry__.smoke()                         -> gpurun_out/TAG_smoke.log
#   bench:WL[:STEPS[:ARGS]]   bench.py line (ARGS: extra flags, ',' for ' ')  -> gpurun_out/TAG_bench_WL.json
#   kstats:WL[:ARGS[:SUF]]    rocprofv3 --kernel-trace --stats, two steps (ARGS: extra bench flags, ',' for ' ';
#                             SUF: suffix of the output names)                -> gpurun_out/TAG_kstats_WL[SUF]/
#   pmc:KERNEL:WL[:sq|hbm]    PMC passes of one kernel (hbm: FETCH_SIZE / WRITE_SIZE passes)
#   ab:WL:BDIR[:STEPS]        same-box ABAB bench lines: this build vs the libraries in BDIR
#   parse[:ROUNDS]            host entropy speed, one thread (tools/parse_bench)
#   prof:WL                   kernel stats + FETCH_SIZE / WRITE_SIZE passes (tools/gpu_prof.sh), summarised by
#                             tools/prof_summary.py into gpurun_out/TAG_WL_summary.md (the roofline `traffic`)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
PKG=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd
for STEP in "$@"; do
  IFS=: read -r KIND A1 A2 A3 <<< "$STEP"
  echo "== $TAG $STEP"
  case $KIND in
  tests)
    K=()
    [ -n "$A1" ] && K=(-k "$A1")
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
      > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
    tail -1 gpurun_out/${TAG}_tests.log ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
      || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
    tail -1 gpurun_out/${TAG}_smoke.log ;;
  bench)
    WL=${A1:-hevc1080}; ST=${A2:-20}; EXTRA=${A3//,/ }
    timeout -k 10 600 python bench.py --gpus 1 --workload $WL --steps $ST --warmup 5 $EXTRA \
      > gpurun_out/${TAG}_bench_$WL.json 2> gpurun_out/${TAG}_bench_$WL.err || { tail -20 gpurun_out/${TAG}_bench_$WL.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('$WL', round(d['value']), 'aim', d.get('value_aim'), 'us/KB', d.get('parse_core_us_per_kb'), 'hbm_res', round(d.get('hbm_resident_fps', 0)), 'frac', d['roofline']['frac'], 'verified', d.get('outputs_verified'))" gpurun_out/${TAG}_bench_$WL.json ;;
  kstats)
    WL=${A1:-hevc1080}; EXTRA=${A2//,/ }; D=gpurun_out/${TAG}_kstats_$WL$A3
    rm -rf $D
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o stats -- \
      python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --no-aim --no-single-call $EXTRA > $D.log 2>&1 \
      || { tail -20 $D.log; exit 1; }
    f=$(find $D -name "*kernel_stats.csv" | head -1)
    cp "$f" gpurun_out/${TAG}_kstats_${WL}$A3.csv
    python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:64].ljust(64), r['Calls'].rjust(6), ('%.3f' % (float(r['AverageNs'])/1e6)).rjust(9), 'ms avg')
" "$f" ;;
  pmc)
    KR=$A1; WL=${A2:-hevc1080}; MODE=${A3:-sq}
    P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
    P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
    if [ "$MODE" = hbm ]; then P1="FETCH_SIZE"; P2="WRITE_SIZE"; fi  # KiB, separate passes (MI355X guide)
    i=0
    for P in "$P1" "$P2"; do
      i=$((i+1)); D=gpurun_out/${TAG}_pmc${i}_$WL
      rm -rf $D
      timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$KR" --output-format csv -d $D -o pmc -- \
        python3 bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline --no-single-call --no-aim > $D.log 2>&1
    done
    python3 - "$TAG" "$WL" <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/{sys.argv[1]}_pmc*_{sys.argv[2]}/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print(f"{k:24s} {acc[k]:16.0f}  (records {n[k]})")
PY
    ;;
  ab)
    WL=${A1:-hevc1080}; BD=$PKG/$A2; ST=${A3:-8}
    for rep in 1 2; do
      for v in A B; do
        if [ $v = A ]; then D=$PKG; else D=$BD; fi
        H2J_LIB_DIR=$D timeout -k 10 300 python bench.py --workload $WL --steps $ST --no-cpu-baseline --no-single-call --no-aim \
          > gpurun_out/${TAG}_ab_${WL}_$v$rep.json 2> gpurun_out/${TAG}_ab_${WL}_$v$rep.err || { tail -5 gpurun_out/${TAG}_ab_${WL}_$v$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_ab_${WL}_$v$rep.json')); k=d['stages_ms_per_step']; print('$WL $v$rep', round(d['value'],1), 'hbm_res', round(d['hbm_resident_fps']), 'k1', round(d['roofline'].get('avg_launch_ms'),3), 'prep', round(k.get('prep_ms',0),3), 'sao', round(k.get('sao_ms',0),3), 'jpeg', round(k.get('jpeg_ms',0),3), 'busy', d['host_cpu_busy_cores'])"
      done
    done ;;
  parse)
    R=${A1:-3}
    timeout -k 10 600 bash tools/gpu_parse_min.sh $R > gpurun_out/${TAG}_parse.log 2>&1 || { tail -20 gpurun_out/${TAG}_parse.log; exit 1; }
    tail -8 gpurun_out/${TAG}_parse.log ;;
  prof)
    WL=${A1:-hevc1080}
    bash tools/gpu_prof.sh ${TAG}_$WL 1024 $WL > /dev/null
    python3 tools/prof_summary.py ${TAG}_$WL $WL > /dev/null
    cp profiles/${TAG}_${WL}_summary.md profiles/${TAG}_${WL}_kernel_stats.csv profiles/pmc_k1_${WL}.json gpurun_out/ 2>/dev/null || true
    head -16 profiles/${TAG}_${WL}_summary.md ;;
  *)
    echo "unknown step $STEP"; exit 2 ;;
  esac
done
