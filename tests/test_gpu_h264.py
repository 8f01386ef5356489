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
