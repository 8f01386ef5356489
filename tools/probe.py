"""Quick timing probe: batch of N copies of a stream through the engine."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h264-h265-to-jpeg_amd"))
import h2j
path = sys.argv[1]; n = int(sys.argv[2]); reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
data = open(path, "rb").read()
eng = h2j.Engine(0)
for r in range(reps):
    t = time.time(); outs = eng.transcode([data] * n); dt = time.time() - t
    st = eng.stats()
    print(f"rep {r}: {n} frames {dt*1e3:.1f} ms -> {n/dt:.1f} fps | " + " ".join(f"{k}={v:.2f}" for k, v in st.items()), flush=True)
assert all(o is not None for o in outs)
