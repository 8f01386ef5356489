"""Diagnostic: GPU pre-loop-filter planes of one HEVC stream against the oracle; prints the
mismatch count per plane and the first mismatching positions (y, x) -> gpurun_out/<tag>_diff.json."""
import json
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, "h264-h265-to-jpeg_amd")
import oracle_py as O  # noqa: E402
from h2j import Engine  # noqa: E402

tag, paths = sys.argv[1], sys.argv[2:]
eng = Engine()
res = {}
for p in paths:
    s = open(p, "rb").read()
    gy, gu, gv, bd = eng.decode(s, stage=1)
    oy, ou, ov, obd = O.decode(s, 265, skip_loop_filter=True)
    r = {}
    for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
        d = np.argwhere(g != o)
        r[name] = {"n": int(len(d)), "first": d[:40].tolist()}
    res[p] = r
    print(p, {k: v["n"] for k, v in r.items()}, flush=True)
json.dump(res, open(f"gpurun_out/{tag}_diff.json", "w"))
