"""GPU parity at the batch sizes bench.py times.

The K1 launch shape depends on the batch: h2j_gpu_predict runs the per-picture kernel up to
128 pictures and the picture pool above, with P = min(4, pictures / 256) pictures per
workgroup (h2j_kernels.hip, h2j_k1_recon_hevc_pool), staged CTB-wide row stores and, at 1080p
CTB64, 17 rows per picture near the 160 KB LDS cap.  These tests run the exact configurations
of BASELINE.json configs[1]-[3]: 1024 hevc1080 pictures (P = 4; the 64-stream §8(d) set and the
lighter round 1-5 set), 1024 avc1080 pictures and 256
hevc2160 Main10 pictures (pool<u16>), through h2j_engine_submit / h2j_engine_wait like the
bench, and compare every JPEG with the oracle's; planes are read from inside bench-sized
batches with h2j_engine_decode_batch (P = 4, P = 3 with a partly filled last workgroup)."""
import glob
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read

pytestmark = pytest.mark.gpu

SETS = {
    "hevc1080": ("bench_aim", "hevc1080a_*.h265", 265, 1024),       # the bench's headline set (r06)
    "hevc1080_light": ("bench", "hevc1080_*.h265", 265, 1024),
    "avc1080": ("bench264", "avc1080_*.h264", 264, 1024),
    "hevc2160": ("bench4k", "hevc2160_10b_*.h265", 265, 256),
}


def _streams(key):
    d, pat, _, _ = SETS[key]
    paths = sorted(glob.glob(os.path.join(golden(d), pat)))
    assert paths, key
    return [read(p) for p in paths]


def _oracle_jpegs(streams):
    with ThreadPoolExecutor(8) as ex:  # ctypes drops the GIL inside the C oracle
        return dict(zip(streams, ex.map(O.transcode, streams)))


@pytest.mark.parametrize("key", sorted(SETS))
def test_bench_sized_batch_every_jpeg(engine, key):
    """configs[1]/[2]/[3] at the bench's own batch: every picture's JPEG == the oracle's."""
    streams = _streams(key)
    n = SETS[key][3]
    batch = [streams[i % len(streams)] for i in range(n)]
    outs = engine.transcode_async([batch])[0]
    ref = _oracle_jpegs(streams)
    bad = [i for i, (s, o) in enumerate(zip(batch, outs)) if o != ref[s]]
    assert not bad, f"{len(bad)} of {n} JPEGs differ, first {bad[:8]}"


@pytest.mark.parametrize("key,n,pick,stage", [
    ("hevc1080", 1024, 1023, 0),   # P = 4, last picture of the last workgroup
    ("hevc1080", 1024, 6, 1),      # P = 4, pre-loop-filter planes
    ("hevc1080", 1022, 1021, 0),   # P = 3, last workgroup holds 2 pictures
    ("hevc1080", 768, 400, 0),     # P = 3
    ("hevc1080_light", 1024, 1000, 0),
    ("hevc2160", 256, 255, 0),     # pool<u16>, 4K Main10
    ("avc1080", 1024, 1023, 0),
])
def test_planes_inside_bench_sized_batch(engine, key, n, pick, stage):
    streams = _streams(key)
    batch = [streams[i % len(streams)] for i in range(n)]
    gy, gu, gv, bd = engine.decode_batch(batch, pick, stage=stage)
    oy, ou, ov, obd = O.decode(batch[pick], SETS[key][2], skip_loop_filter=stage == 1)
    assert bd == obd
    for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
        diff = np.argwhere(g != o)
        assert diff.size == 0, f"{name}: {len(diff)} mismatches, first {diff[:4].tolist()}"


def test_payload_copy_across_buffer_growth():
    """r05: the JPEG payloads follow the kernels in-stream, sized by the slot's pinned buffer; a
    chunk whose payload outgrows it is copied again whole after the host reads the total.  A fresh
    engine (empty buffers) goes small -> large -> small, sequentially and pipelined, and every JPEG
    must still equal the oracle's."""
    import h2j
    small = [read(golden("img01.h265"))]
    large = _streams("hevc1080")
    ref = _oracle_jpegs(small + large)
    eng = h2j.Engine(0)
    plan = [small * 4, large[:8] * 8, small * 16, large * 4]
    for batch in plan:  # one chunk per call: each slot sees the growth on its own buffer
        outs = eng.transcode(batch)
        assert all(o == ref[s] for s, o in zip(batch, outs)), "sequential"
    fresh = h2j.Engine(0)
    outs_all = fresh.transcode_async(plan)
    for batch, outs in zip(plan, outs_all):
        bad = [i for i, (s, o) in enumerate(zip(batch, outs)) if o != ref[s]]
        assert not bad, f"pipelined: {len(bad)} of {len(batch)} differ"
