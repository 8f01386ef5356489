# r03l: host parse on the box CPU: thread scaling (parse_bench 1/8/16 threads) and a sampling
# profile of the single-thread HEVC parse (pb_sample, tools/parse_bench/sample_report.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_parse_mt.sh
cd tools/parse_bench
H2J_SAMPLE_OUT=$GRAFT_REPO_ROOT/gpurun_out/samples_hevc.txt ./pb_sample ../../tests/golden/bench/*.h265 -r 20
H2J_SAMPLE_OUT=$GRAFT_REPO_ROOT/gpurun_out/samples_hevc16.txt ./pb_sample ../../tests/golden/bench/*.h265 -r 64 -t 16
python3 sample_report.py pb_sample $GRAFT_REPO_ROOT/gpurun_out/samples_hevc.txt 40 > $GRAFT_REPO_ROOT/gpurun_out/r03l_sample_hevc.txt
python3 sample_report.py pb_sample $GRAFT_REPO_ROOT/gpurun_out/samples_hevc16.txt 40 > $GRAFT_REPO_ROOT/gpurun_out/r03l_sample_hevc16.txt
head -50 $GRAFT_REPO_ROOT/gpurun_out/r03l_sample_hevc.txt
