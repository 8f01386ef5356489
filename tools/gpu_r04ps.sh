# r04ps: sampling profile of the single-thread HEVC parse on the box CPU after the r04p engine
# changes (pb_sample built with -DH2J_SAMPLE, report by tools/parse_bench/sample_report.py).
cd $GRAFT_REPO_ROOT/tools/parse_bench
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
H2J_SAMPLE_OUT=$GRAFT_REPO_ROOT/gpurun_out/samples_r04ps.txt ./pb_sample ../../tests/golden/bench/*.h265 -r 20
