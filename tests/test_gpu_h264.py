"""GPU parity of the H.264 path against the oracle (pinned on img01.h264)."""
import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read

pytestmark = pytest.mark.gpu


def _cmp(g, o, what):
    for a, b, name in zip(g, o, "YUV"):
        diff = np.argwhere(a != b)
        assert diff.size == 0, f"{what} {name}: {len(diff)} mismatches, first {diff[:4].tolist()}"


def test_h264_pre_deblock_bit_exact(engine):
    s = read(golden("img01.h264"))
    gy, gu, gv, _ = engine.decode(s, stage=1)
    oy, ou, ov, _ = O.decode(s, 264, skip_loop_filter=True)
    _cmp((gy, gu, gv), (oy, ou, ov), "pre-deblock")


def test_h264_decoded_bit_exact(engine):
    s = read(golden("img01.h264"))
    gy, gu, gv, _ = engine.decode(s, stage=0)
    oy, ou, ov, _ = O.decode(s, 264)
    _cmp((gy, gu, gv), (oy, ou, ov), "final")


def test_h264_transcode_matches_fixture(engine):
    s = read(golden("img01.h264"))
    assert engine.transcode([s])[0] == read(golden("img01.h264.jpeg"))


import glob
import os

H264_DIR = golden("h264")
# h264wide: wider than the deblocking kernel's LDS line buffer (global line buffer path)
PARITY264 = sorted(glob.glob(os.path.join(H264_DIR, "*.h264"))) + sorted(glob.glob(os.path.join(golden("h264wide"), "*.h264")))


@pytest.mark.parametrize("path", PARITY264, ids=[os.path.basename(p) for p in PARITY264])
def test_h264_parity_vectors(engine, path):
    """h264gen vectors: Main/High/High10, I8x8, PCM, slices, QP deltas,
    chroma QP offsets, deblocking offsets and disable_deblocking_filter_idc; 6144- and
    8192-wide pictures."""
    s = read(path)
    for stage, skip in ((1, True), (0, False)):
        gy, gu, gv, bd = engine.decode(s, stage=stage)
        oy, ou, ov, obd = O.decode(s, 264, skip_loop_filter=skip)
        assert bd == obd
        _cmp((gy, gu, gv), (oy, ou, ov), f"stage {stage}")


def test_h264_mixed_codec_batch(engine):
    """H.264 and H.265 pictures in one batch; every JPEG byte-exact."""
    streams = [read(p) for p in PARITY264] + [read(golden("img01.h264")), read(golden("img01.h265"))]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, PARITY264 + ["img01.h264", "img01.h265"]):
        assert o is not None, p
        assert o == O.transcode(s), p


def test_h264_bench_streams_sample(engine):
    paths = sorted(glob.glob(os.path.join(golden("bench264"), "*.h264")))[::5]
    streams = [read(p) for p in paths]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, paths):
        assert o == O.transcode(s), p


TALL264 = [golden("mixed/avc2160_00.h264")] + sorted(glob.glob(os.path.join(golden("h264tall"), "*.h264")))


@pytest.mark.parametrize("path", TALL264, ids=[os.path.basename(p) for p in TALL264])
def test_h264_tall_picture_banded(engine, path):
    """Pictures taller than 68 MB rows (engine.cpp kK1BandRows) run h2j_k1_recon_h264 in 8-row
    bands, one 8-wave workgroup each, dispatched band-major, and the deblocking in 16-row bands,
    both handing boundary rows across workgroups through the xline buffer: 3840x2160 (135 MB rows:
    17 K1 bands, the last 7 rows; 9 deblocking bands), a 10-bit 256x1152 (72 rows: 9 K1 bands of
    8, h264_rows<uint16_t>; 5 deblocking bands) and an 8-bit CAVLC 192x1408 (88 rows: 11 / 6)."""
    s = read(path)
    for stage, skip in ((1, True), (0, False)):
        gy, gu, gv, bd = engine.decode(s, stage=stage)
        oy, ou, ov, obd = O.decode(s, 264, skip_loop_filter=skip)
        assert bd == obd
        _cmp((gy, gu, gv), (oy, ou, ov), f"stage {stage}")


def test_h264_tall_pictures_one_batch(engine):
    """Banded pictures of three heights and two sample types in one batch (shared band-major K1
    map, per-picture xline regions); every JPEG byte-exact."""
    streams = [read(p) for p in TALL264] + [read(TALL264[1])]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, TALL264 + TALL264[1:2]):
        assert o is not None, p
        assert o == O.transcode(s), p


def test_mixed_workload_batch(engine):
    """configs[4] sample: 720p H.264/H.265 and banded 2160p H.264 in one batch."""
    paths = sorted(glob.glob(os.path.join(golden("mixed"), "*")))
    streams = [read(p) for p in paths]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, paths):
        assert o == O.transcode(s), p


def test_merged_k1_launch_mixed_kinds(engine):
    """A batch of more than 128 pictures mixing HEVC 8-bit, HEVC 10-bit (incl. a 4K
    picture on 16-wave groups) and H.264 (incl. a banded 4K picture) runs K1 as one
    merged launch (h2j_k1_recon_any); every JPEG byte-exact."""
    hevc = sorted(glob.glob(os.path.join(golden("hevc"), "*.h265")))
    tall = [sorted(glob.glob(os.path.join(golden("bench4k"), "*.h265")))[0], golden("mixed/avc2160_00.h264")]
    kinds = [read(p) for p in tall + PARITY264 + hevc]  # 4K HEVC: 16-wave groups; 4K H.264: bands
    assert any("10bit" in p for p in hevc)
    streams = [kinds[i % len(kinds)] for i in range(160)]
    want = {i: O.transcode(s) for i, s in enumerate(kinds)}
    outs = engine.transcode(streams)
    for i, o in enumerate(outs):
        assert o == want[i % len(kinds)], i
