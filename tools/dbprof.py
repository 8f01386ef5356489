"""Raw cycle buckets of the instrumented kernels (-DH2J_PROF build) for N frames of
one stream; see the PROF_LAP / PROF_LAPK calls in h2j_kernels.hip for the bucket map."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-h265-to-jpeg_amd")
os.environ["H2J_LIB_DIR"] = os.path.join(PKG, "build", os.environ.get("H2J_PROF_VARIANT", "prof"))
sys.path.insert(0, PKG)
import h2j
path, n = sys.argv[1], int(sys.argv[2])
eng = h2j.Engine(0)
hip = ctypes.CDLL(os.path.join(os.environ["H2J_LIB_DIR"], "libh2j_hip.so"))
buf = (ctypes.c_ulonglong * 16)()
data = open(path, "rb").read()
eng.transcode([data] * 4)
hip.h2j_gpu_prof(buf, 16, 1)
eng.transcode([data] * n)
st = eng.stats()
hip.h2j_gpu_prof(buf, 16, 1)
v = list(buf)
units = max(1, v[6])
print(f"{os.path.basename(path)} x{n}: deblock {st['deblock_ms']:.2f} ms recon {st['recon_ms']:.2f} ms units {units}")
for i in range(16):
    if i not in (4, 6, 7):
        print(f"  [{i:2d}] {v[i] / units:10.0f} cyc/unit")
if v[4]:
    print(f"  clock {100.0 * v[7] / v[4]:.0f} MHz")
