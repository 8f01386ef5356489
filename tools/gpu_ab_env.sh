# Same-box A/B of an environment switch on bench lines (K1 ms, hbm_resident fps):
#   gpurun -- bash tools/gpu_ab_env.sh TAG VAR "V1 V2 ..." WL[,WL...] [STEPS]
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; VAR=$2; VALS=$3; WLS=$4; ST=${5:-4}
for rep in 1 2; do
  for WL in ${WLS//,/ }; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python3 bench.py --workload $WL --steps $ST --warmup 1 --no-cpu-baseline --no-single-call --no-aim \
        > gpurun_out/${TAG}_${WL}_${v}_$rep.json 2> gpurun_out/${TAG}_${WL}_${v}_$rep.err || { tail -5 gpurun_out/${TAG}_${WL}_${v}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['stages_ms_per_step']; print('$WL $VAR=$v rep $rep', 'k1', round(d['roofline']['avg_launch_ms'],3), 'hbm_res', round(d['hbm_resident_fps']), 'value', round(d['value']), 'kern', {k: round(st[k],2) for k in ('prep_ms','recon_ms','deblock_ms','sao_ms','jpeg_ms','entropy_ms')})" gpurun_out/${TAG}_${WL}_${v}_$rep.json
    done
  done
done
