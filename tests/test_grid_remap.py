"""The XCD-aware workgroup order the K0 / SAO / K4c / K5b / K5d grids use
(h264-h265-to-jpeg_amd/csrc/hip/grid.h, xcd_remap) is a bijection of the launch's
workgroup ids for every grid size, and gives each of the 8 XCD groups (orig % 8)
one contiguous id range.  The header's own function is compiled with g++ on the
host (no GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR_DIR = os.path.join(ROOT, "h264-h265-to-jpeg_amd", "csrc", "hip")

SRC = r"""
#include <cstdio>
#include <vector>
#include "grid.h"
int main() {
    const unsigned sizes[] = {1, 7, 8, 9, 15, 16, 17, 255, 256, 257, 510, 768, 1000, 48960, 522240};
    for (unsigned n : sizes) {
        std::vector<unsigned char> seen(n, 0);
        std::vector<unsigned> lo(8, ~0u), hi(8, 0), cnt(8, 0);
        for (unsigned o = 0; o < n; o++) {
            const unsigned id = xcd_remap(o, n);
            if (id >= n || seen[id]) { std::printf("FAIL n=%u orig=%u id=%u\n", n, o, id); return 1; }
            seen[id] = 1;
            const unsigned g = o & 7u;
            lo[g] = id < lo[g] ? id : lo[g];
            hi[g] = id > hi[g] ? id : hi[g];
            cnt[g]++;
        }
        for (unsigned g = 0; g < 8; g++)
            if (cnt[g] && hi[g] - lo[g] + 1 != cnt[g]) { std::printf("FAIL n=%u group %u not contiguous\n", n, g); return 1; }
    }
    std::printf("ok\n");
    return 0;
}
"""


def test_xcd_remap_is_a_bijection_with_contiguous_xcd_ranges(tmp_path):
    src = tmp_path / "grid_remap.cpp"
    src.write_text(SRC)
    exe = tmp_path / "grid_remap"
    try:
        subprocess.check_call(["g++", "-std=c++11", "-O1", "-I", HDR_DIR, str(src), "-o", str(exe)])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.fail(f"g++ could not build the grid.h check: {e}")
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip() == "ok"
