"""Per-kind cost of the configs[4] mixed batch's K1: transcodes subsets of
bench.py's 1024-picture mixed list as single 1024-or-fewer-picture launches, so that
`rocprofv3 --kernel-trace --stats` shows what each kind costs in its own launch against the
merged `h2j_k1_recon_any` of the whole list.

    H2J_CHUNK=1024 H2J_TAIL=0 rocprofv3 --kernel-trace --stats -d DIR -o stats -- \\
        python3 tools/mixed_k1_probe.py SUBSET

SUBSET: all | hevc | h264 | hevc_small (720p + 1080p HEVC) | hevc_4k | h264_small | h264_4k |
no_h264_4k | no_hevc_4k.
Every output is checked against tests/golden/bench_manifest.json's md5 of its stream.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "h264-h265-to-jpeg_amd"))

import bench  # noqa: E402  (mixed_list: the bench's own configs[4] list)
import h2j  # noqa: E402


def main():
    subset = sys.argv[1] if len(sys.argv) > 1 else "all"
    items = bench.mixed_list(1024)
    keep = []
    for g, it in enumerate(items):
        cls = "720" if g % 10 < 4 else ("1080" if g % 10 < 8 else "2160")
        codec = 265 if (g // 10) % 2 == 0 else 264
        ok = {
            "all": True,
            "hevc": codec == 265,
            "h264": codec == 264,
            "hevc_small": codec == 265 and cls != "2160",
            "hevc_4k": codec == 265 and cls == "2160",
            "h264_small": codec == 264 and cls != "2160",
            "h264_4k": codec == 264 and cls == "2160",
            "no_h264_4k": not (codec == 264 and cls == "2160"),
            "no_hevc_4k": not (codec == 265 and cls == "2160"),
        }[subset]
        if ok:
            keep.append(it[0])
    manifest = json.load(open(os.path.join(ROOT, "tests/golden/bench_manifest.json")))
    known = {k: v["jpeg_md5"] for k, v in manifest.items()}  # stream md5 -> JPEG md5
    eng = h2j.Engine(0)
    bad = 0
    for _ in range(2):
        outs = eng.transcode(keep)
        for s, o in zip(keep, outs):
            want = known.get(hashlib.md5(s).hexdigest())
            if o is None or want is None or hashlib.md5(o).hexdigest() != want:
                bad += 1
    print(json.dumps({"subset": subset, "pictures": len(keep), "bad": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
