"""CPU: the oracle's demux handles the Annex-B variants identically (the same
checks run on the GPU path in test_gpu_annexb.py)."""
import pytest

import oracle_py as O
from annexb_variants import variants
from conftest import golden, read

CASES = [("img01.h265", 265), ("img01.h264", 264), ("hevc/p03_400x232_pcm_bypass_slices.h265", 265),
         ("h264/a15_352x288_cavlc_high8x8_pcm.h264", 264)]


@pytest.mark.parametrize("name,codec", CASES, ids=[c[0].split("/")[-1] for c in CASES])
def test_oracle_annexb_variants(name, codec):
    s = read(golden(name))
    ref = O.transcode(s)
    for vname, v in variants(s, codec).items():
        assert O.transcode(v) == ref, vname
