"""GPU: Annex-B wire-format variants transcode to the original's JPEG."""
import pytest

import oracle_py as O
from annexb_variants import variants
from conftest import golden, read

pytestmark = pytest.mark.gpu

CASES = [("img01.h265", 265), ("img01.h264", 264), ("hevc/p03_400x232_pcm_bypass_slices.h265", 265),
         ("h264/a15_352x288_cavlc_high8x8_pcm.h264", 264)]


@pytest.mark.parametrize("name,codec", CASES, ids=[c[0].split("/")[-1] for c in CASES])
def test_gpu_annexb_variants(engine, name, codec):
    s = read(golden(name))
    ref = O.transcode(s)
    vs = variants(s, codec)
    outs = engine.transcode(list(vs.values()))
    for (vname, _), o in zip(vs.items(), outs):
        assert o == ref, vname
