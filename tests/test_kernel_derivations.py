"""CPU: the restatements two round-6 kernels rely on, checked exhaustively on the host.

* HEVC K0's availability masks in closed form (h2j_k0_prep, pictures without slices / tiles) equal the
  per-unit rule on every aligned TB position of 8..200 x 8..136 pictures at CTB 16 / 32 / 64.
* K4c's AP-922 FDCT on column pairs (fdct_ap922_pk: wrapping int16 halves, rows by dot2) equals the
  saturating scalar form on 4 M random and extreme blocks of samples in [0, 255].

These check the arithmetic the kernels restate; the GPU parity suite checks the kernels themselves."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(src, tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "chk")
    subprocess.check_call(["g++", "-O2", "-o", exe, os.path.join(ROOT, "tools", "diag", src)])
    return subprocess.run([exe], capture_output=True, text=True, timeout=300, check=True).stdout


def test_k0_mask_closed_form(tmp_path):
    out = _run("k0_mask_check.cpp", tmp_path)
    assert "0 mismatches" in out and "971658 cases" in out, out


def test_fdct_column_pairs(tmp_path):
    out = _run("fdct_pk_check.cpp", tmp_path)
    assert "mismatches 0" in out, out
    assert int(out.split("max |intermediate|")[1]) <= 32767, out
