"""The C++ drop-in surface: a program written against the reference's
IDecoder.h (README.md:38-54 usage) links libH265ToJpeg.so and transcodes."""
import os
import subprocess

import pytest

from conftest import golden, read

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-h265-to-jpeg_amd")

DRIVER = r'''
#include "IDecoder.h"
#include <cstdio>
int main(int argc, char** argv) {
    auto decoder = IDecoder::getInstance();
    if (!decoder) return 3;
    bool ok = decoder->H265ToJpeg(argv[1], argv[2]);
    bool bad = IDecoder::getInstance()->H265ToJpeg("", argv[2]);
    return ok && !bad ? 0 : 1;
}
'''


def test_idecoder_cpp_driver(tmp_path):
    src = tmp_path / "drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.check_call(["g++", "-std=c++11", "-O1", str(src), "-I", os.path.join(ROOT, "include"), "-L", PKG,
                           "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    out = tmp_path / "out.jpg"
    r = subprocess.run([str(exe), golden("img01.h265"), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import oracle_py as O
    assert out.read_bytes() == O.transcode(read(golden("img01.h265")))


def test_python_h265_to_jpeg(tmp_path):
    import h2j
    out = tmp_path / "o.jpg"
    assert h2j.h265_to_jpeg(golden("img01.h265"), str(out))
    assert not h2j.h265_to_jpeg(str(tmp_path / "missing.h265"), str(out))
