"""GPU parity of the HEVC path against the oracle (and through it the
reference's fixtures).  Integer work: bit-exact everywhere."""
import hashlib

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read

pytestmark = pytest.mark.gpu


def test_prelf_recon_bit_exact(engine):
    s = read(golden("img01.h265"))
    gy, gu, gv, bd = engine.decode(s, stage=1)
    oy, ou, ov, _ = O.decode(s, 265, skip_loop_filter=True)
    for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
        diff = np.argwhere(g != o)
        assert diff.size == 0, f"{name}: {len(diff)} mismatches, first at {diff[:5].tolist()}"


def test_decoded_picture_bit_exact(engine):
    s = read(golden("img01.h265"))
    gy, gu, gv, _ = engine.decode(s, stage=0)
    oy, ou, ov, _ = O.decode(s, 265)
    for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
        diff = np.argwhere(g != o)
        assert diff.size == 0, f"{name}: {len(diff)} mismatches, first at {diff[:5].tolist()}"


def test_jpeg_coefficients_exact(engine):
    s = read(golden("img01.h265"))
    qs, co = engine.jpeg_coeffs(s)
    oy, ou, ov, bd = O.decode(s, 265)
    oqs, oco = O.jpeg_coeffs(O.to8(oy, bd), O.to8(ou, bd), O.to8(ov, bd))
    assert qs == oqs
    assert np.array_equal(co, oco)


def test_transcode_matches_fixture(engine):
    s = read(golden("img01.h265"))
    out = engine.transcode([s])[0]
    ref = read(golden("img01.h265.jpeg"))
    # golden carries the mac build's COM ('Lavc58.91.100'); compare after it
    def strip_com(j):
        assert j[2:4] == b"\xff\xfe"
        n = (j[4] << 8) | j[5]
        return j[:2] + j[4 + n:]
    assert strip_com(out) == strip_com(ref)
    assert out == O.transcode(s)
