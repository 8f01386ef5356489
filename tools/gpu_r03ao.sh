# r03ao: no K4a launch when K3 SAO has summed every picture's MB variances (h2j_gpu_batch.k4a_frames;
# hevc1080): GPU JPEG parity, then same-box A/B against build/base.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_h264.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
WLS="hevc1080" VARIANTS="nok4a:.: base:build/base:" REPS=3 bash tools/gpu_k1ab.sh
