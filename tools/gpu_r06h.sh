# GPU CABAC feasibility probe: one wave per stream decoding a dependent chain of
# context-coded bins; ns per bin per wave and aggregate bins/s at 1..8192 waves
set -e
cd "$GRAFT_REPO_ROOT/tools/gpu_cabac_probe"
mkdir -p ../../gpurun_out
timeout -k 10 300 ./cabac_probe ../../tests/golden/bench_aim/hevc1080a_00.h265 | tee ../../gpurun_out/r06v_cabac_probe.txt
