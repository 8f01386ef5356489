"""Expected-output manifest for bench.py's post-timing check.

For every stream bench.py can put in a batch (tests/golden/{bench,bench_aim,bench_heavy,bench264,bench4k,
mixed}), records md5(stream bytes) -> md5(oracle JPEG) in tests/golden/bench_manifest.json.
bench.py hashes the JPEGs of its last timed step after the timed region and reports
"outputs_verified".  The oracle (test infrastructure) runs only here, when minting; bench.py
reads the JSON file only.

    python tools/make_bench_manifest.py
"""
import glob
import hashlib
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402

SETS = ["bench/*.h265", "bench_aim/*.h265", "bench_heavy/*.h265", "bench264/*.h264", "bench264_heavy/*.h264", "bench4k/*.h265", "mixed/*.h26[45]"]


def main():
    files = sorted(f for p in SETS for f in glob.glob(os.path.join(ROOT, "tests", "golden", p)))
    streams = [open(f, "rb").read() for f in files]
    with ThreadPoolExecutor(8) as ex:  # ctypes drops the GIL inside the C oracle
        jpegs = list(ex.map(O.transcode, streams))
    man = {}
    for f, s, j in zip(files, streams, jpegs):
        man[hashlib.md5(s).hexdigest()] = {"file": os.path.relpath(f, os.path.join(ROOT, "tests", "golden")),
                                           "jpeg_md5": hashlib.md5(j).hexdigest(), "jpeg_bytes": len(j)}
    out = os.path.join(ROOT, "tests", "golden", "bench_manifest.json")
    json.dump(man, open(out, "w"), indent=1, sort_keys=True)
    print(f"{out}: {len(man)} streams")


if __name__ == "__main__":
    main()
