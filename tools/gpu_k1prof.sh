# K1 cycle accounting (-DH2J_PROF build in build/prof) over a few streams, 1024 pictures each
# through the asynchronous path (the bench's launch shape).  gpurun -- bash tools/gpu_k1prof.sh TAG FILE...
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
shift
for f in "$@"; do
  K1PROF_ASYNC=1 timeout -k 10 200 python3 tools/k1prof.py "$f" 1024 >> gpurun_out/${TAG}_k1prof.txt 2>&1 || { tail -5 gpurun_out/${TAG}_k1prof.txt; exit 1; }
done
cat gpurun_out/${TAG}_k1prof.txt
