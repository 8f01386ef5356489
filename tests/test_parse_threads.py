"""Intra-picture parallel parsing: pictures with several
independent slices decode them on several host threads, and a single WPP
(entropy_coding_sync) slice decodes its CTB rows side by side from the entry
points, and a single tiled slice its tiles; the records must be identical to a single-threaded parse (parse_bench
output digest)."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "h264-h265-to-jpeg_amd", "csrc", "host")


@pytest.fixture(scope="module")
def parse_bench(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pb") / "parse_bench")
    srcs = [os.path.join(ROOT, "tools", "parse_bench", "parse_bench.cpp")] + [
        os.path.join(HOST, f) for f in ("bitstream.cpp", "cabac_tables.cpp", "hevc_parser.cpp", "h264_parser.cpp")]
    subprocess.check_call(["g++", "-O1", "-std=c++11", "-pthread", "-I", os.path.join(ROOT, "include"), "-I", HOST]
                          + srcs + ["-o", exe])
    return exe


def _digest(exe, path, threads):
    out = subprocess.check_output([exe, path, "-r", "1", "-d", "-p", str(threads)], text=True)
    return out.split()[-1] if "digest" in out.splitlines()[0] else out.splitlines()[0].split()[-1]


MULTI = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "h264", "*slices*.h264")) +
               glob.glob(os.path.join(ROOT, "tests", "golden", "hevc", "*slices*.h265")) +
               glob.glob(os.path.join(ROOT, "tests", "golden", "hevc", "*wpp*.h265")) +
               glob.glob(os.path.join(ROOT, "tests", "golden", "hevc", "p18_*tiles*.h265")))


@pytest.mark.parametrize("path", MULTI, ids=[os.path.basename(p) for p in MULTI])
def test_slice_parallel_parse_is_identical(parse_bench, path):
    assert len(MULTI) >= 12
    one = _digest(parse_bench, path, 1)
    assert _digest(parse_bench, path, 8) == one
    assert _digest(parse_bench, path, 2) == one


# Record digests of the benchmark sets as the round-4 parser produced them before its speed work
# (0784438; DESIGN.md §6 "Round 4: host entropy"): engine / residual-loop changes must leave every
# TU, coefficient, CTB and slice record bit-identical.
PINNED = {
    "bench": "f9d574ef25e13d13",
    "bench_heavy": "46d227bd85837eb8",
    "bench264": "03609146691cbedd",
    "bench4k": "c2630db4567d8cfa",
}


@pytest.mark.parametrize("name", sorted(PINNED))
def test_parse_records_pinned(parse_bench, name):
    paths = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", name, "*.h26?")))
    assert len(paths) >= 4
    out = subprocess.check_output([parse_bench] + paths + ["-r", "1", "-d"], text=True)
    assert out.split()[-1] == PINNED[name]
