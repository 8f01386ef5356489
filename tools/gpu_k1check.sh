# K1 change check: GPU parity suite, K1 per launch size on hevc1080 / hevc2160, then K1 cycle
# accounting of the pooled kernel (make prof build) at 512 pictures (P = 2).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_k1.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_k1.log | head -30; tail -30 gpurun_out/pt_k1.log; exit 1; }
tail -1 gpurun_out/pt_k1.log
b() {  # label, env, bench args
  env $2 timeout -k 10 300 python bench.py $3 --no-cpu-baseline --no-single-call --no-aim > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']; print('$1', round(d['value'],1), 'hbm_fps', round(d['hbm_resident_fps'],1), 'K1/step', round(d['stages_ms_per_step']['recon_ms'],2), 'frac', round(r['frac'],4), 'parse', round(d['stages_ms_per_step']['parse_ms'],1), {k:(v['avg_k1_ms'],v['frac']) for k,v in r['per_launch_size'].items()})"
}
b "hevc async" "H2J_K1_POOL=4" "--workload hevc1080 --steps 6"
b "4k async" "" "--workload hevc2160 --frames 256 --steps 3"
timeout -k 10 60 python3 -u tools/k1prof.py tests/golden/bench/hevc1080_00.h265 512 > gpurun_out/k1prof512.log 2>&1
cat gpurun_out/k1prof512.log
