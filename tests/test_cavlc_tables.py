"""CPU: the H.264 CAVLC VLC tables.  The product parser and tools/h264gen share the tables
tools/gen_cavlc_tables.py generates (h264-h265-to-jpeg_amd/csrc/host/cavlc_tables.h); the
oracle uses its own hand-typed copy in the layout of the reference's decoder, FFmpeg
h264_cavlc.c (oracle/cavlc_spec.h).  Every entry of the two typings must agree, and every
table of the hand-typed copy must be a prefix code (ITU-T H.264 Tables 9-4, 9-5, 9-7, 9-8,
9-9(a), 9-10)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "h264-h265-to-jpeg_amd/csrc/host/cavlc_tables.h")
GEN2 = os.path.join(ROOT, "tools/h264gen/cavlc_tables.h")
SPEC = os.path.join(ROOT, "oracle/cavlc_spec.h")


def c_arrays(path):
    """name -> nested list of ints for every `static const T name[..]... = {...};`"""
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"static const \w+ (\w+)((?:\[[^\]]*\])+)\s*=\s*(\{.*?\});", text, flags=re.S):
        dims = [eval(d) for d in re.findall(r"\[([^\]]*)\]", m.group(2))]
        body = m.group(3).replace("{", "[").replace("}", "]")
        val = eval(body)

        def pad(v, dims):  # C zero-fills short initialisers
            if not dims:
                return v
            v = list(v) + [0 if len(dims) == 1 else []] * (dims[0] - len(v))
            return [pad(x, dims[1:]) for x in v]
        out[m.group(1)] = pad(val, dims)
    return out


G = c_arrays(GEN)
S = c_arrays(SPEC)


def test_generated_copies_identical():
    assert open(GEN).read() == open(GEN2).read()


def prefix_free(codes):
    """codes: list of (len, value); True if no code is a prefix of another, plus the Kraft sum"""
    words = [format(v, "0%db" % n) for n, v in codes]
    for i, a in enumerate(words):
        for j, b in enumerate(words):
            if i != j and b.startswith(a):
                return False, None
    return True, sum(2.0 ** -len(w) for w in words)


def test_coeff_token_equal():
    for cls in range(3):
        for tc in range(17):
            for t1 in range(4):
                i = tc * 4 + t1
                assert G["kCoeffTokenLen"][cls][t1][tc] == S["k_ct_len"][cls][i], (cls, tc, t1)
                if S["k_ct_len"][cls][i]:
                    assert G["kCoeffTokenCode"][cls][t1][tc] == S["k_ct_bits"][cls][i], (cls, tc, t1)
    for tc in range(5):
        for t1 in range(4):
            i = tc * 4 + t1
            assert G["kCoeffTokenLen"][3][t1][tc] == S["k_ct_dc_len"][i], ("dc", tc, t1)
            if S["k_ct_dc_len"][i]:
                assert G["kCoeffTokenCode"][3][t1][tc] == S["k_ct_dc_bits"][i], ("dc", tc, t1)


def test_total_zeros_run_before_cbp_equal():
    for k in range(15):
        for z in range(17 - (k + 1)):
            assert G["kTotalZerosLen"][k][z] == S["k_tz_len"][k][z], (k, z)
            assert G["kTotalZerosCode"][k][z] == S["k_tz_bits"][k][z], (k, z)
    for k in range(3):
        for z in range(4 - k):
            assert G["kTotalZerosDcLen"][k][z] == S["k_tz_dc_len"][k][z]
            assert G["kTotalZerosDcCode"][k][z] == S["k_tz_dc_bits"][k][z]
    for k in range(7):
        for r in range(k + 2 if k < 6 else 15):
            assert G["kRunBeforeLen"][k][r] == S["k_run_len"][k][r], (k, r)
            assert G["kRunBeforeCode"][k][r] == S["k_run_bits"][k][r], (k, r)
    assert G["kCbpIntra"] == S["k_cbp_intra"]
    assert sorted(S["k_cbp_intra"]) == list(range(48))


@pytest.mark.parametrize("cls", [0, 1, 2, "dc"])
def test_coeff_token_prefix_codes(cls):
    if cls == "dc":
        lens, bits = S["k_ct_dc_len"], S["k_ct_dc_bits"]
    else:
        lens, bits = S["k_ct_len"][cls], S["k_ct_bits"][cls]
    codes = [(n, v) for n, v in zip(lens, bits) if n]
    ok, kraft = prefix_free(codes)
    assert ok
    # 62 codes (17 x 4 less the impossible T1s > TotalCoeff); Table 9-5 leaves only the
    # all-zero words of the longest lengths unused
    assert len(codes) == (62 if cls != "dc" else 14)
    assert kraft <= 1.0
    assert kraft > 0.99


def test_total_zeros_and_run_before_prefix_codes():
    for k in range(15):
        codes = [(S["k_tz_len"][k][z], S["k_tz_bits"][k][z]) for z in range(16 - k)]
        ok, kraft = prefix_free(codes)
        # complete but for tzVlcIndex 1, whose all-zero 9-bit word is unused
        assert ok and kraft == (1.0 if k else 1.0 - 2.0 ** -9), k
    for k in range(3):
        codes = [(S["k_tz_dc_len"][k][z], S["k_tz_dc_bits"][k][z]) for z in range(4 - k)]
        ok, kraft = prefix_free(codes)
        assert ok and kraft == 1.0, k
    for k in range(7):
        n = k + 2 if k < 6 else 15
        codes = [(S["k_run_len"][k][r], S["k_run_bits"][k][r]) for r in range(n)]
        ok, kraft = prefix_free(codes)
        assert ok, k
        assert kraft <= 1.0
