"""GPU: SURVEY.md §8 f3 wire-format edge cases and malformed parameter sets.

f3 vectors (tests/golden/f3, tools/make_streams.py f3): decoder-delay streams (VUI
max_num_reorder_frames / sps_max_num_reorder_pics > 0, then reordered all-skip P pictures)
and leading non-IDR I / CRA / BLA pictures.  The reference returns false without output for
the decoder-delay ones (/root/reference/src/Decoder.cpp:342-360: one packet sent, no flush,
avcodec_receive_frame gives EAGAIN); this build transcodes picture 0 (INTEGRATION.md,
"Documented differences") -- its planes and JPEG must equal the oracle's.

With H2J_STRICT_REFERENCE=1 the engine returns no JPEG for the decoder-delay streams, as the
reference does, and keeps transcoding every other vector.

Malformed vectors (tests/golden/malformed): HEVC conformance windows that leave no picture are
ignored as FFmpeg's hevc_ps.c ignores them (a JPEG of the whole coded picture, equal to the
oracle's); H.264 cropping that leaves no picture fails as h264_ps.c rejects the SPS; the other
vectors fail cleanly with a per-picture message."""
import json
import os

import numpy as np
import pytest

import oracle_py as O
from annexb_variants import variants
from conftest import golden, read

pytestmark = pytest.mark.gpu

F3 = json.load(open(golden("f3/manifest.json")))
BAD = json.load(open(golden("malformed/manifest.json")))


@pytest.mark.parametrize("e", F3, ids=[e["file"] for e in F3])
def test_f3_picture0_planes_and_jpeg(engine, e):
    s = read(golden("f3/" + e["file"]))
    for stage, skip in ((1, True), (0, False)):
        gy, gu, gv, bd = engine.decode(s, stage=stage)
        oy, ou, ov, obd = O.decode(s, e["codec"], skip_loop_filter=skip)
        assert bd == obd
        for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
            assert np.array_equal(g, o), f"stage {stage} {name}"
    ref = O.transcode(s)
    vs = variants(s, e["codec"])
    outs = engine.transcode([s] + list(vs.values()))
    assert outs[0] == ref
    for (vname, _), o in zip(vs.items(), outs[1:]):
        assert o == ref, vname


def test_malformed_parameter_sets(engine):
    streams = [read(golden("malformed/" + e["file"])) for e in BAD]
    outs = engine.transcode(streams)
    for i, (e, s, o) in enumerate(zip(BAD, streams, outs)):
        if e["expect"] == "ok":
            assert o is not None, (e["file"], engine.frame_error(i))
            assert o == O.transcode(s), e["file"]
            assert engine.frame_error(i) == ""
        else:
            assert o is None, e["file"]
            assert engine.frame_error(i), e["file"]  # a per-picture message, not the engine-wide one
            if "message" in e:
                assert e["message"] in engine.frame_error(i), (e["file"], engine.frame_error(i))


def test_strict_reference_mode_on_decoder_delay_streams(engine):
    """H2J_STRICT_REFERENCE=1: false (no JPEG, a per-picture message) exactly where the reference
    returns false (/root/reference/src/Decoder.cpp:342-360); the default engine transcodes them."""
    import h2j
    streams = [read(golden("f3/" + e["file"])) for e in F3]
    default = engine.transcode(streams)
    os.environ["H2J_STRICT_REFERENCE"] = "1"
    try:
        strict_engine = h2j.Engine()
    finally:
        del os.environ["H2J_STRICT_REFERENCE"]
    strict = strict_engine.transcode(streams)
    for i, (e, d, st) in enumerate(zip(F3, default, strict)):
        assert d is not None and d[:2] == b"\xff\xd8", e["file"]
        if e["reference_returns"] is False:
            assert st is None, e["file"]
            assert "decoder delay" in strict_engine.frame_error(i), e["file"]
        else:
            assert st == d, e["file"]


def test_strict_reference_mode_on_field_pairs(engine):
    """PAFF field pairs (tests/golden/h264/a37-a40): the default engine outputs the frame FFmpeg
    outputs after the second field (bit-exact to the oracle in test_gpu_h264.py); with
    H2J_STRICT_REFERENCE=1 it returns no JPEG, as the reference does for a field picture (one packet
    holds one field, /root/reference/src/Decoder.cpp:324, 342-360)."""
    import glob
    import h2j
    paths = sorted(glob.glob(golden("h264/*_paff_*.h264")))
    assert len(paths) >= 4
    streams = [read(p) for p in paths]
    default = engine.transcode(streams)
    os.environ["H2J_STRICT_REFERENCE"] = "1"
    try:
        strict_engine = h2j.Engine()
    finally:
        del os.environ["H2J_STRICT_REFERENCE"]
    strict = strict_engine.transcode(streams)
    for i, (p, d, st) in enumerate(zip(paths, default, strict)):
        assert d is not None and d == O.transcode(streams[i]), p
        assert st is None, p
        assert "field picture" in strict_engine.frame_error(i), p
