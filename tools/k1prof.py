"""K1 cycle accounting: run N frames of a stream through the -DH2J_PROF build
and print where the K1 waves spend their cycles (s_memtime, shader clock).
  make -C h264-h265-to-jpeg_amd prof && python tools/k1prof.py tests/golden/bench/hevc1080_00.h265 256"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-h265-to-jpeg_amd")
os.environ["H2J_LIB_DIR"] = os.path.join(PKG, "build", os.environ.get("H2J_PROF_VARIANT", "prof"))
# the cycle counters cover every HEVC K1 kernel, the picture pool (default, H2J_K1_POOL=4) included
sys.path.insert(0, PKG)
import h2j
files = [a for a in sys.argv[1:] if not a.isdigit()]
n = int([a for a in sys.argv[1:] if a.isdigit()][0]) if any(a.isdigit() for a in sys.argv[1:]) else 256
eng = h2j.Engine(0)
hip = ctypes.CDLL(os.path.join(os.environ["H2J_LIB_DIR"], "libh2j_hip.so"))
buf = (ctypes.c_ulonglong * 16)()
for path in files:
    data = open(path, "rb").read()
    t0 = time.time()
    eng.transcode([data] * 8)
    print(f"warm-up done {time.time() - t0:.1f}s", flush=True)
    hip.h2j_gpu_prof(buf, 16, 1)
    # K1PROF_ASYNC=1: through the asynchronous path (one chunk of up to 1024 pictures)
    outs = eng.transcode_async([[data] * n])[0] if os.environ.get("K1PROF_ASYNC") else eng.transcode([data] * n)
    bad = [i for i, o in enumerate(outs) if o is None]
    if bad:
        print(f"{len(bad)} pictures failed, e.g. {eng.frame_error(bad[0])!r}", flush=True)
        sys.exit(1)
    print(f"batch done {time.time() - t0:.1f}s", flush=True)
    st = eng.stats()
    if hip.h2j_gpu_prof(buf, 16, 1) != 0:
        print(f"not a -DH2J_PROF build (K1 {st['recon_ms']:.2f} ms)")
        continue
    v = list(buf)
    waves = None
    tot = sum(v[0:4]) + sum(v[8:16])
    ntu, nctb = v[5], v[6]
    print(f"{os.path.basename(path)}: {n} frames, K1 {st['recon_ms']:.2f} ms, TUs {ntu}, CTBs {nctb}")
    if path.endswith((".h264", ".264")) and os.environ.get("K1PROF_AVCK1"):
        # H.264 K1 (build with PROFDEFS="-DH2J_PROF -DH2J_PROF_AVCK1"), per macroblock
        print(f"  MBs {nctb}, TUs {ntu}")
        for i, nm in enumerate(["wait", "window", "tb-setup", "store"]):
            print(f"  {nm:10s} {v[i] / max(1, nctb):10.0f} cyc/MB  {100 * v[i] / tot:5.1f}%")
        for k, nm in enumerate(["I4x4", "I8x8", "I16x16", "I4x4 DC", "I8x8 DC", "I16x16 DC", "chroma", "-"]):
            print(f"  {nm:10s} {v[8 + k] / max(1, nctb):10.0f} cyc/MB  {100 * v[8 + k] / tot:5.1f}%")
        continue
    if path.endswith((".h264", ".264")):
        # H.264: the counters are the K2 deblock wave's (h264_db_rows), per macroblock
        names = ["wait", "window", "params", "store"]
        for i, nm in enumerate(names):
            print(f"  {nm:8s} {v[i] / max(1, nctb):10.0f} cyc/MB  {100 * v[i] / tot:5.1f}%")
        for k, nm in ((0, "V edges"), (4, "H edges")):
            print(f"  {nm:8s} {v[8 + k] / max(1, nctb):10.0f} cyc/MB  {100 * v[8 + k] / tot:5.1f}%")
        continue
    names = ["wait", "setup", "-", "store"]
    for i, nm in enumerate(names):
        if i != 2:
            print(f"  {nm:8s} {v[i] / max(1, nctb):10.0f} cyc/CTB  {100 * v[i] / tot:5.1f}%")
    for k in range(8):
        print(f"  {'YC'[k // 4]} {4 << (k % 4):2d}x{4 << (k % 4):<2d} {v[8 + k] / max(1, nctb):10.0f} cyc/CTB  {100 * v[8 + k] / tot:5.1f}%")
    print(f"  TU loop {sum(v[8:16]) / max(1, ntu):.0f} cyc/TU")
    if v[4]:
        print(f"  s_memtime rate vs 100 MHz s_memrealtime: {100.0 * v[7] / v[4]:.0f} MHz (shader clock)")
