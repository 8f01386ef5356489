# r03al: K4c occupancy bounds 6 / 7 waves per SIMD (build/k6, build/k7) against the release build
# (94 VGPRs, 5 waves): JPEG parity on each variant (HEVC suite), then same-box A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in k6 k7; do
  H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/$v timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -2
done
WLS="hevc1080 avc1080" VARIANTS="k6:build/k6: k7:build/k7: base:.:" REPS=2 bash tools/gpu_k1ab.sh
