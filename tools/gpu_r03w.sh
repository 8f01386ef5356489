# r03w: HEVC K1 pool job order: a row index's luma rows of all P pictures, then their chroma rows
# (build/jobb) against (picture, luma, chroma) interleaving (release): HEVC parity on the variant
# build, then same-box A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H2J_LIB_DIR=$GRAFT_REPO_ROOT/h264-h265-to-jpeg_amd/build/jobb timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="hevc1080" VARIANTS="jobb:build/jobb: base:.:" REPS=3 bash tools/gpu_k1ab.sh
