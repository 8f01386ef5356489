# r03x: HEVC K1 pool job order: chroma rows one row index behind the luma rows (build/jobd)
# against luma-then-chroma per row index (release): HEVC parity on the variant
# build, then same-box A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/jobd timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="hevc1080" VARIANTS="jobd:build/jobd: base:.:" REPS=3 bash tools/gpu_k1ab.sh
