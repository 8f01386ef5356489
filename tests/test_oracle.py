"""Pins the ORACLE against the reference's own fixtures (test/img/*, copied
to tests/golden/) and the known-answer values of SURVEY.md Appendix B.
CPU only."""
import hashlib

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read

# SURVEY.md Appendix B (outputs of the reference's FFmpeg path in the survey container)
H265_YUV = ("2c57d662215a27330b512584b1b6e154", "a61ade531310678e34e8b281d08c2dcf", "f14fbd3733c3b6cf75983eb06a439356")
H265_PRELF = ("e2f95f4b56f328c1725d40c7c3ff84bf", "4b7e7ac57262ef60e36a2c393ed6602c", "a3e41b507587956d8525e0d2ef73ec4a")
H264_YUV = ("163d91eb322b1e75acc6362edb06464e", "b2828e5be85105f2a5688e7ae2798185", "b57b4ed32ca0b4c414ff91b2cc934eb0")
H264_PRELF = ("81a6e9b53b03c9fe042761d738b16c40", "1af126324c7c95c5a03bc95cc607fa2a", "b0755d1f501cdcbb1cc53e0491c3b95f")


def md5_planes(planes):
    return tuple(hashlib.md5(p.astype(np.uint8).tobytes()).hexdigest() for p in planes)


@pytest.mark.parametrize("name,com", [("img01.h264.jpeg", b"Lavc58.117.101"), ("img01.h265.jpeg", b"Lavc58.91.100")])
def test_huffman_reemission_byte_exact(name, com):
    """Parse the fixture JPEG's coefficients and re-emit: optimal Huffman
    (package-merge + AV_QSORT order) and bitstream must be byte-identical."""
    jpg = read(golden(name))
    w, h, dqt, coefs = O.jpeg_parse(jpg)
    qscale = dqt[1] // 2
    out = O.jpeg_from_coeffs(coefs, w, h, qscale, com)
    assert out == jpg


def test_hevc_decode_matches_appendix_b():
    y, u, v, bd = O.decode(read(golden("img01.h265")), 265)
    assert (y.shape, bd) == ((1440, 2560), 8)
    assert md5_planes((y, u, v)) == H265_YUV


def test_hevc_pre_loop_filter_matches_appendix_b():
    y, u, v, _ = O.decode(read(golden("img01.h265")), 265, skip_loop_filter=True)
    assert md5_planes((y, u, v)) == H265_PRELF


def test_hevc_transcode_matches_fixture_jpeg():
    """Full reference behaviour: decode + RC + FDCT + quant + Huffman.  The
    golden was written by the mac build (COM 'Lavc58.91.100')."""
    out = O.transcode(read(golden("img01.h265")), b"Lavc58.91.100")
    assert out == read(golden("img01.h265.jpeg"))


def test_fdct_dc_and_flat_block():
    import ctypes
    blk = (ctypes.c_int16 * 64)(*([128] * 64))
    O.lib().oracle_fdct(blk)
    # flat block: only DC, level 128 after ((X>>2)+8)/16
    assert ((blk[0] >> 2) + 8) // 16 == 128


def test_h264_decode_matches_appendix_b():
    y, u, v, bd = O.decode(read(golden("img01.h264")), 264)
    assert (y.shape, bd) == ((1080, 1920), 8)
    assert md5_planes((y, u, v)) == H264_YUV


def test_h264_pre_deblock_matches_appendix_b():
    y, u, v, _ = O.decode(read(golden("img01.h264")), 264, skip_loop_filter=True)
    assert md5_planes((y, u, v)) == H264_PRELF


def test_h264_transcode_matches_fixture_jpeg():
    """The golden img01.h264.jpeg was written by the x86_64 build: byte-exact,
    COM 'Lavc58.117.101' included."""
    assert O.transcode(read(golden("img01.h264"))) == read(golden("img01.h264.jpeg"))


def test_oracle_mono_chroma_is_half_range():
    """4:0:0 H.264 (tests/golden/h264/a41..a45): FFmpeg decodes into yuv420p with every chroma
    sample 1 << (BitDepth - 1) (DC_128 prediction, I_PCM memset), so the oracle's chroma planes are
    flat at that value (parity unpinned: no reference-held monochrome fixture)."""
    import glob
    import os
    for p in sorted(glob.glob(golden("h264/a4[1-5]_*mono*.h264"))):
        y, u, v, bd = O.decode(read(p), 264)
        assert (u == 1 << (bd - 1)).all() and (v == 1 << (bd - 1)).all(), os.path.basename(p)
        assert y.std() > 1.0  # a real luma picture
