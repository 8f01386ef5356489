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


import glob
import json
import os

HEVC_DIR = golden("hevc")
PARITY = sorted(glob.glob(os.path.join(HEVC_DIR, "*.h265")))


@pytest.mark.parametrize("path", PARITY, ids=[os.path.basename(p) for p in PARITY])
def test_parity_vectors_prelf_and_final(engine, path):
    """hevcgen vectors (PCM, bypass, slices, 10-bit, CTB16/32, offsets, SDH, scaling lists, WPP, tiles,
    9 / 12 bits, RExt tools; r06: p33-p39 -- extended_precision_processing and cabac_bypass_alignment
    decoded as FFmpeg 4.3 decodes them (as if 0), CU chroma QP offsets with lists of 1 / 2 / 3 / 6
    entries at group depths 0-3, in the Cb / Cr dequantisation QP only).  Pre-loop-filter and final
    planes equal the oracle's (parity unpinned against the reference for the RExt vectors)."""
    s = read(path)
    for stage, skip in ((1, True), (0, False)):
        gy, gu, gv, bd = engine.decode(s, stage=stage)
        oy, ou, ov, obd = O.decode(s, 265, skip_loop_filter=skip)
        assert bd == obd
        for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
            diff = np.argwhere(g != o)
            assert diff.size == 0, f"stage {stage} {name}: {len(diff)} mismatches, first {diff[:4].tolist()}"


def test_mixed_batch_transcode_matches_oracle(engine):
    """One batch mixing sizes, bit depths and features; every JPEG byte-exact."""
    streams = [read(p) for p in PARITY] + [read(golden("img01.h265"))]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, PARITY + ["img01"]):
        assert o is not None, p
        assert o == O.transcode(s), p


def test_bench_streams_sample(engine):
    paths = sorted(glob.glob(os.path.join(golden("bench"), "*.h265")))[::5]
    streams = [read(p) for p in paths]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, paths):
        assert o == O.transcode(s), p


def test_bench_nosdh_1080p(engine):
    """configs[1]-sized pictures with sign-data hiding off (tools/make_streams.py nosdh): the path
    the reference fixture img01.h265 pins, at 1080p; planes and JPEG equal the oracle's."""
    paths = sorted(glob.glob(os.path.join(golden("bench_nosdh"), "*.h265")))
    assert len(paths) == 2
    streams = [read(p) for p in paths]
    outs = engine.transcode(streams)
    for s, o, p in zip(streams, outs, paths):
        assert o == O.transcode(s), p
        gy, gu, gv, bd = engine.decode(s, stage=0)
        oy, ou, ov, obd = O.decode(s, 265)
        for g, q, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
            assert np.array_equal(g, q), (p, name)


def test_high_entropy_tiles_both_emit_paths(engine):
    """tiles over kEmitWords words take K5d's global-memory path beside LDS-path tiles
    (tests/test_entropy_vectors.py proves the vectors straddle the limit); H2J_EMIT_GLOBAL=1 puts
    every tile on the global path.  Every JPEG byte-exact against the oracle on both."""
    paths = sorted(glob.glob(os.path.join(golden("entropy"), "*.h265")))
    streams = [read(p) for p in paths] + [read(p) for p in PARITY[:6]] + [read(golden("img01.h265"))]
    refs = [O.transcode(s) for s in streams]
    assert engine.transcode(streams) == refs
    os.environ["H2J_EMIT_GLOBAL"] = "1"
    try:
        assert engine.transcode(streams) == refs
    finally:
        del os.environ["H2J_EMIT_GLOBAL"]


def test_invalid_inputs_fail_cleanly(engine):
    outs = engine.transcode([b"", b"\x00\x00\x01\x40garbage", read(golden("img01.h265"))[:1000]])
    assert outs[0] is None and outs[1] is None


def test_4k_main10_stream(engine):
    """configs[3]: 3840x2160 Main10 -> 10-bit decode bit-exact, 8-bit JPEG byte-exact."""
    path = sorted(glob.glob(os.path.join(golden("bench4k"), "*.h265")))[0]
    s = read(path)
    gy, gu, gv, bd = engine.decode(s, stage=0)
    oy, ou, ov, obd = O.decode(s, 265)
    assert bd == obd == 10
    for g, o, name in ((gy, oy, "Y"), (gu, ou, "U"), (gv, ov, "V")):
        assert np.array_equal(g, o), name
    assert engine.transcode([s])[0] == O.transcode(s)


def test_async_batches_and_pooled_k1(engine):
    """h2j_engine_submit / h2j_engine_wait with three batches in flight.  Batches over 256 pictures
    run K1's picture pool (h2j_k1_recon_hevc_pool) with P = min(4, pictures // 256) pictures per
    workgroup: 520 pictures -> 2 per workgroup, 300 -> 1 (tests/test_gpu_benchsize.py covers
    P = 3 and 4 at the bench's sizes); 8-bit and 10-bit parity vectors (two pool launches),
    scaling lists, PCM, tiles, WPP.  A mixed-codec batch takes the merged K1 launch."""
    streams = [read(p) for p in PARITY]
    h264 = [read(p) for p in sorted(glob.glob(os.path.join(golden("h264"), "*.h264")))]
    big = (streams * 30)[:520]
    mixed = [x for pair in zip(streams * 8, h264 * 8) for x in pair][:300]
    batches = [big, streams[:7], big[:300], mixed]
    outs = engine.transcode_async(batches)
    ref = {s: O.transcode(s) for s in set(streams) | set(h264)}
    for b_in, b_out in zip(batches, outs):
        assert len(b_in) == len(b_out)
        for k, (s, o) in enumerate(zip(b_in, b_out)):
            assert o == ref[s], k
    assert engine.transcode([streams[0]])[0] == ref[streams[0]]  # the synchronous path still works
