"""The CPU baseline (bench.cpu_baseline) runs the oracle on several host threads at once:
concurrent transcodes must give the same bytes as one after another (no shared mutable
state in oracle/: package-merge lists are per thread, tables set up once)."""
import glob
import os
import sys
import threading

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py  # noqa: E402


def test_concurrent_oracle_transcodes_match_sequential():
    files = (sorted(glob.glob(os.path.join(ROOT, "tests/golden/hevc/p0*.h265")))[:4]
             + sorted(glob.glob(os.path.join(ROOT, "tests/golden/h264/a0*.h264")))[:4])
    assert files
    streams = [open(f, "rb").read() for f in files]
    want = [oracle_py.transcode(s) for s in streams]
    got = [None] * (2 * len(streams))

    def run(i):
        got[i] = oracle_py.transcode(streams[i % len(streams)])

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(got))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i, g in enumerate(got):
        assert g == want[i % len(streams)], files[i % len(streams)]


def test_bench_cpu_baseline_reports_threads():
    sys.path.insert(0, ROOT)
    import bench
    streams = [open(f, "rb").read() for f in sorted(glob.glob(os.path.join(ROOT, "tests/golden/hevc/*.h265")))[:4]]
    r = bench.cpu_baseline(streams, 3, budget_s=0.5)
    assert r["cores"] == 3 and r["kind"] == "port" and r["value"] > 0


@pytest.mark.gpu
def test_bench_single_call_latency_through_mem_entry():
    """bench.single_call_latency (configs[0]) goes through h2j_h265_to_jpeg_mem, the IDecoder
    engine: the JPEG it returns equals the oracle's for the reference fixture."""
    sys.path.insert(0, ROOT)
    import bench
    fx = open(os.path.join(ROOT, "tests/golden/img01.h265"), "rb").read()
    r = bench.single_call_latency([("img01.h265", fx)], calls=1)
    assert r["img01.h265"] > 0
    import ctypes
    import h2j
    lib = h2j.load_library()
    jp = ctypes.POINTER(ctypes.c_uint8)()
    jl = ctypes.c_size_t()
    buf = (ctypes.c_uint8 * len(fx)).from_buffer_copy(fx)
    assert lib.h2j_h265_to_jpeg_mem(buf, len(fx), ctypes.byref(jp), ctypes.byref(jl)) == 0
    got = ctypes.string_at(jp, jl.value)
    lib.h2j_free(jp)
    assert got == oracle_py.transcode(fx)
