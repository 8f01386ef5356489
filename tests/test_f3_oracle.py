"""CPU: the oracle on the f3 and malformed vectors (the GPU path is checked against the same
expectations in test_gpu_f3.py).  For f3 vectors the oracle's pre-loop-filter decode of
picture 0 equalled the generator's reconstruction when they were minted
(tools/make_streams.py f3); the trailing P pictures of the decoder-delay streams are never
decoded (only picture 0 is used, /root/reference/src/Decoder.cpp:342-355)."""
import json

import pytest

import oracle_py as O
from annexb_variants import variants
from conftest import golden, read

F3 = json.load(open(golden("f3/manifest.json")))
BAD = json.load(open(golden("malformed/manifest.json")))


@pytest.mark.parametrize("e", F3, ids=[e["file"] for e in F3])
def test_oracle_f3(e):
    s = read(golden("f3/" + e["file"]))
    ref = O.transcode(s)
    assert ref[:2] == b"\xff\xd8"
    for vname, v in variants(s, e["codec"]).items():
        assert O.transcode(v) == ref, vname


@pytest.mark.parametrize("e", BAD, ids=[e["file"] for e in BAD])
def test_oracle_malformed(e):
    s = read(golden("malformed/" + e["file"]))
    if e["expect"] == "ok":
        j = O.transcode(s)
        assert j[:2] == b"\xff\xd8"
    else:
        with pytest.raises(RuntimeError):
            O.transcode(s)
