"""Benchmark: 1080p H.265 I-frames/s -> JPEG on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): a batch of 1024 x 1080p H.265 Main 8-bit
I-frames -> baseline JPEG on one GPU.  Inputs are the 64 committed hevcgen
streams of tests/golden/bench_aim (SURVEY.md §8(d) recipe: QP {22,27,32,37},
seeded crops / flips of the fixture content + noise, 110-220 KB per picture)
tiled x16; every frame is decoded independently (no dedupe).  The lighter
16-stream set of rounds 1-5 (tests/golden/bench, 72 KB per picture) is
reported beside it as value_light.

One step = one full transcode of the batch: host entropy threads
(CABAC -> job records), H2D, the HIP pixel pipeline (K1 recon, K2 deblock,
K3 SAO, K4 JPEG forward path), D2H, host Huffman assembly.  `value` is the
whole-job frames/s; the GPU-pipeline-only rate and the per-stage times are
reported beside it.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): one process per GPU,
each transcodes its own 1024-frame batch (weak scaling, no data-path
collective); a barrier brackets the timed region and rank 0 reports the max
time over ranks.  The only collectives are the counter reductions at the end.
"""
import argparse
import ctypes
import glob
import json
import resource
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "h264-h265-to-jpeg_amd"))

METRIC = "1080p H.265 I-frames/sec → JPEG at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)
# algorithmic bytes per frame B = 5S, S = 1.5*W*H*bytes_per_sample
WORKLOADS = {
    "hevc1080": dict(streams="tests/golden/bench_aim/hevc1080a_*.h265", w=1920, h=1080, bps=1,
                     desc="configs[1]: batch of 1024 x 1080p H.265 Main 8-bit I-frames -> JPEG per GPU",
                     data="64 distinct hevcgen 1080p HEVC Main I-frame streams, QP {22,27,32,37}, 110-220 KB per "
                          "picture (SURVEY.md §8(d) configs[1] recipe, tests/golden/bench_aim)"),
    "hevc1080_light": dict(streams="tests/golden/bench/hevc1080_*.h265", w=1920, h=1080, bps=1,
                           desc="configs[1] on the lighter round 1-5 set (~72 KB per picture): batch of 1024 x "
                                "1080p H.265 Main 8-bit I-frames -> JPEG per GPU",
                           data="16 hevcgen 1080p HEVC Main I-frame streams, QP {22,27,32,37} x noise {0,2,4} "
                                "(tests/golden/bench)"),
    "avc1080": dict(streams="tests/golden/bench264/avc1080_*.h264", w=1920, h=1080, bps=1,
                    desc="configs[2]: batch of 1024 x 1080p H.264 High (8x8 transform) I-frames -> JPEG per GPU",
                    data="16 h264gen 1080p H.264 High I-frame streams, 2/16 CAVLC (SURVEY.md §8(d) mix: "
                         "avc1080_07 / _15) (tests/golden/bench264)"),
    "hevc2160": dict(streams="tests/golden/bench4k/hevc2160_10b_*.h265", w=3840, h=2160, bps=2,
                     desc="configs[3]: 4K H.265 Main10 I-frames, 10-bit decode -> 8-bit JPEG per GPU",
                     data="4 hevcgen 2160p HEVC Main10 I-frame streams (tests/golden/bench4k)"),
    "hevc1080_heavy": dict(streams="tests/golden/bench_heavy/hevc1080h_*.h265", w=1920, h=1080, bps=1,
                           desc="configs[1] on heavier streams (~100-250 KB per picture, SURVEY.md §8(d) aim): "
                                "batch of 1024 x 1080p H.265 Main 8-bit I-frames -> JPEG per GPU",
                           data="16 hevcgen 1080p HEVC Main I-frame streams, QP 18-24, noise sigma 0-2 (tests/golden/bench_heavy)"),
    "avc1080_heavy": dict(streams="tests/golden/bench264_heavy/avc1080h_*.h264", w=1920, h=1080, bps=1,
                          desc="configs[2] on heavier streams (~75-230 KB per picture, SURVEY.md §8(d) aim): "
                               "batch of 1024 x 1080p H.264 High I-frames -> JPEG per GPU",
                          data="16 h264gen 1080p H.264 High I-frame streams, QP 18-24, noise sigma 0-1, 2/16 CAVLC "
                               "(tests/golden/bench264_heavy)"),
    "mixed": dict(streams=None, w=None, h=None, bps=None,
                  desc="configs[4]: mixed 720p/1080p/4K (40/40/20 by count) x H.264/H.265 (50/50) stills, "
                       "LPT-sharded over the GPUs (frames = per-GPU share of the global list)",
                  data="tests/golden/{mixed,bench,bench264,bench4k} generator streams"),
}

# configs[4] ingredients: (size class, codec) -> (glob, w, h, bytes/sample)
MIXED_SETS = {
    ("720", 265): ("tests/golden/mixed/hevc720_*.h265", 1280, 720, 1),
    ("720", 264): ("tests/golden/mixed/avc720_*.h264", 1280, 720, 1),
    ("1080", 265): ("tests/golden/bench/hevc1080_*.h265", 1920, 1080, 1),
    ("1080", 264): ("tests/golden/bench264/avc1080_*.h264", 1920, 1080, 1),
    ("2160", 265): ("tests/golden/bench4k/hevc2160_10b_*.h265", 3840, 2160, 2),
    ("2160", 264): ("tests/golden/mixed/avc2160_*.h264", 3840, 2160, 1),
}


def alg_bytes(w, h, bps):
    """B = 2S (int16 residual in) + bps*S (picture out) + 2S (int16 JPEG coefficients out)."""
    return (4 + bps) * (w * h * 3 // 2)


def alg_bytes_per_frame(wl):
    return alg_bytes(wl["w"], wl["h"], wl["bps"])


def mixed_list(total):
    """Deterministic configs[4] list: index g -> size class by g % 10 (0-3 720p,
    4-7 1080p, 8-9 4K), codec by (g // 10) % 2, stream by (g // 20)."""
    sets = {k: (load_streams(v[0]), v[1], v[2], v[3]) for k, v in MIXED_SETS.items()}
    items = []
    for g in range(total):
        cls = "720" if g % 10 < 4 else ("1080" if g % 10 < 8 else "2160")
        codec = 265 if (g // 10) % 2 == 0 else 264
        streams, w, h, bps = sets[(cls, codec)]
        items.append((streams[(g // 20) % len(streams)], alg_bytes(w, h, bps), w * h, bps))
    return items


def load_streams(pattern):
    files = sorted(glob.glob(os.path.join(ROOT, pattern)))
    if not files:
        raise SystemExit(f"no benchmark streams at {pattern}: run tools/make_streams.py bench")
    return [open(f, "rb").read() for f in files]


def pmc_traffic(workload):
    """HBM bytes per K1 launch from the committed rocprofv3 PMC summary
    (profiles/pmc_k1_<workload>.json, written by tools/prof_summary.py), if any."""
    path = os.path.join(ROOT, "profiles", f"pmc_k1_{workload}.json")
    if os.path.exists(path):
        try:
            return json.load(open(path)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            return None
    return None


def reduce_over_ranks(dist, elapsed, frames, local_rank=0):
    """The run's only collectives: MAX of the timed region, SUM of the frames
    (RCCL over xGMI on GPUs, gloo on CPU).  Returns (elapsed, total_frames)."""
    if dist is None:
        return elapsed, frames
    import torch
    use_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
    dev = torch.device("cuda", local_rank) if use_gpu else torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([frames], dtype=torch.int64, device=dev)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), int(c.item())


def sum_over_ranks(dist, value, local_rank=0):
    """SUM of an integer counter over ranks (the output-check mismatch count)."""
    if dist is None:
        return value
    import torch
    use_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
    dev = torch.device("cuda", local_rank) if use_gpu else torch.device("cpu")
    c = torch.tensor([value], dtype=torch.int64, device=dev)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return int(c.item())


def verify_outputs(batch, out, offs, lens, manifest):
    """After the timed region: md5 of every JPEG of one step against tests/golden/bench_manifest.json
    (md5(stream) -> md5 of the oracle's JPEG, minted by tools/make_bench_manifest.py).  Returns
    (pictures checked, mismatches, streams missing from the manifest)."""
    import hashlib
    mv = memoryview(out)
    smd5 = {}
    bad = missing = 0
    for i, b in enumerate(batch):
        key = smd5.get(id(b))
        if key is None:
            key = smd5[id(b)] = hashlib.md5(b).hexdigest()
        ent = manifest.get(key)
        if ent is None:
            missing += 1
            continue
        if hashlib.md5(mv[offs[i]:offs[i] + lens[i]]).hexdigest() != ent["jpeg_md5"]:
            bad += 1
    return len(batch), bad, missing


def shard_lpt(costs, world):
    """Size-balanced LPT partition of independent stills over `world` GPUs
    (SURVEY.md §8e, config 5): returns one index list per rank."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    loads = [0.0] * world
    parts = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        parts[r].append(i)
        loads[r] += costs[i]
    return [sorted(p) for p in parts]


def rank_batch(workload, frames, world, rank):
    """This rank's share of the job: (indices into the global list, global list).

    Uniform workloads: every rank transcodes its own `frames`-picture batch (weak scaling).
    configs[4] (mixed): the global list of frames * world stills (65,536 at --frames 8192 on
    8 GPUs) is LPT-sharded by estimated cost (bitstream bytes for the host CABAC/CAVLC +
    pixels for the GPU), so the shards are disjoint, complete and balanced."""
    if workload != "mixed":
        return list(range(frames)), None
    items = mixed_list(frames * world)
    return shard_lpt([len(b) + 0.02 * px for b, _, px, _ in items], world)[rank], items


# The reference's own CPU path (FFmpeg git-2021-01-28-6fd0116 through IDecoder), measured in the
# survey container (8 vCPU Xeon) -- a different machine from the GPU box, where the
# reference's prebuilt FFmpeg libraries may not run; reported beside the oracle port, labelled.
REFERENCE_CONTAINER = {
    "where": "survey container, 8 vCPU Intel Xeon (BASELINE.md) -- not this box",
    "h264_1080p_img01_ms_per_img_1core": 51.1,
    "h264_1080p_img01_no_probe_ms_1core": 31.4,
    "h264_1080p_img01_img_per_s_8proc": 66.8,
    "hevc_1440p_img01_ms_per_img_1core": 127.3,
    "hevc_1440p_img01_no_probe_ms_1core": 69.3,
    "hevc_1440p_img01_img_per_s_8proc": 55.5,
}


def cpu_baseline(streams, threads, budget_s=12.0):
    """Oracle (CPU restatement of the reference path) on the host cores this rank's GPU
    path uses (`threads`, SURVEY.md §8(d): T threads, one transcode each at a time), on a
    bounded sample: the workload's distinct streams round-robin for about budget_s.
    ctypes drops the GIL for the C call, so the threads run the C oracle in parallel."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py  # test infrastructure: only the cpu_baseline leg uses it
    oracle_py.transcode(streams[0])  # one-time table set-up outside the clock
    lat = []
    for _ in range(3):  # single-call latency on one core (the reference's own per-call figure)
        t = time.perf_counter()
        oracle_py.transcode(streams[0])
        lat.append((time.perf_counter() - t) * 1e3)
    lock = threading.Lock()
    state = {"next": 0, "done": 0}
    t0 = time.perf_counter()

    def worker():
        while time.perf_counter() - t0 < budget_s:
            with lock:
                i = state["next"]
                state["next"] += 1
            oracle_py.transcode(streams[i % len(streams)])
            with lock:
                state["done"] += 1

    pool = [threading.Thread(target=worker) for _ in range(max(1, threads))]
    for t in pool:
        t.start()
    for t in pool:
        t.join()
    dt = time.perf_counter() - t0
    n = state["done"]
    return {"value": n / dt, "unit": "frames/s", "cores": max(1, threads), "kind": "port",
            "single_call_ms": round(sorted(lat)[1], 2),
            "reference_container": REFERENCE_CONTAINER,
            "sample": f"{n} transcodes of the {len(streams)} distinct benchmark streams (round-robin, "
                      f"~{budget_s:.0f} s), oracle decode+JPEG, {max(1, threads)} threads"}


def single_call_latency(streams, calls=9):
    """configs[0]: one still per call through the in-memory IDecoder entry point
    (h2j_h265_to_jpeg_mem, the same process-wide engine IDecoder::H265ToJpeg uses, minus the
    file I/O).  Median wall ms per call after two warm-up calls; a lone call gets the whole
    host pool for its slices / WPP rows / tiles."""
    import h2j
    lib = h2j.load_library()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    lib.h2j_h265_to_jpeg_mem.restype = ctypes.c_int
    lib.h2j_h265_to_jpeg_mem.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
    lib.h2j_free.argtypes = [ctypes.c_void_p]
    res = {}
    for name, s in streams:
        buf = (ctypes.c_uint8 * len(s)).from_buffer_copy(s)
        ms = []
        for i in range(calls + 2):
            jp = u8p()
            jl = ctypes.c_size_t()
            t = time.perf_counter()
            rc = lib.h2j_h265_to_jpeg_mem(buf, len(s), ctypes.byref(jp), ctypes.byref(jl))
            dt = (time.perf_counter() - t) * 1e3
            if rc != 0:
                raise RuntimeError(f"h2j_h265_to_jpeg_mem failed rc={rc} on {name}")
            lib.h2j_free(jp)
            if i >= 2:
                ms.append(dt)
        res[name] = round(sorted(ms)[len(ms) // 2], 2)
    return res


def timed_batches(eng, batch, steps, warmup):
    """Frames/s of `steps` pipelined 1024-picture steps (after `warmup`) of `batch` on `eng`, the
    same submit/wait pattern as the main measurement; returns (fps, per-step stats)."""
    n = len(batch)
    bufs = [(ctypes.c_uint8 * len(s)).from_buffer_copy(s) for s in batch]
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    sizes = (ctypes.c_size_t * n)(*[len(s) for s in batch])
    cap = n * (2 << 20)
    outsets = [((ctypes.c_uint8 * cap)(), (ctypes.c_size_t * n)(), (ctypes.c_size_t * n)(), (ctypes.c_int * n)())
               for _ in range(2)]
    acc = {}

    def run(k_steps, record):
        inflight = []
        for k in range(k_steps + 1):
            if k < k_steps:
                out, offs, lens, status = outsets[k % 2]
                inflight.append((eng.submit_raw(ptrs, sizes, n, out, cap, offs, lens, status), status))
            if k > 0:
                t, status = inflight.pop(0)
                if eng.wait(t) != 0 or any(status[i] != 0 for i in range(n)):
                    raise RuntimeError(f"transcode failed: {eng.error()}")
                if record:
                    for key, v in eng.stats().items():
                        acc[key] = acc.get(key, 0.0) + v

    run(warmup, False)
    t0 = time.perf_counter()
    run(steps, True)
    dt = time.perf_counter() - t0
    return n * steps / dt, {k: v / steps for k, v in acc.items()}


def parse_core_us_per_kb(per, threads, batch):
    """Host entropy cost: the pool's wall time on a batch (first to last picture parsed) x its
    threads, per KB of bitstream."""
    return round(per["parse_run_ms"] * 1e3 * threads / (sum(len(b) for b in batch) / 1024), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (r06: 12 timed steps after 2 warmup steps by default -- with two batches in flight the
    # first step of a timed region carries the pipeline fill; 6 steps read a few % under 20)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1024, help="frames per GPU per step")
    ap.add_argument("--threads", type=int, default=0,
                    help="host entropy/Huffman threads per GPU (default: the engine's NUMA-local share, "
                         "include/h2j.h h2j_engine_create)")
    ap.add_argument("--workload", default="hevc1080", choices=sorted(WORKLOADS),
                    help="hevc1080 = the BASELINE metric's config; the others are configs[2]/[3]/[4]")
    ap.add_argument("--streams", default=None, help="override the workload's stream glob")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync", action="store_true",
                    help="one synchronous h2j_engine_transcode per step (no cross-step overlap)")
    ap.add_argument("--no-single-call", action="store_true",
                    help="skip the configs[0] single-call latencies (profiling runs: no extra 1-picture launches)")
    ap.add_argument("--no-aim", action="store_true",
                    help="skip value_aim (configs[1] on the 100-250 KB/picture set) and the host-thread sweep")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        tdist.init_process_group(backend=backend)
        dist = tdist

    import h2j
    wl = WORKLOADS[args.workload]
    n = args.frames
    mine, items = rank_batch(args.workload, n, world, rank)
    if args.workload == "mixed":
        batch = [items[i][0] for i in mine]
        frame_bytes = [items[i][1] for i in mine]
        frame_bps = [items[i][3] for i in mine]
        streams = sorted({id(b): b for b in batch}.values(), key=len)
        n = len(batch)
    else:
        streams = load_streams(args.streams or wl["streams"])
        batch = [streams[i % len(streams)] for i in range(n)]
        frame_bytes = [alg_bytes_per_frame(wl)] * n
        frame_bps = [wl["bps"]] * n
    # host pool: the engine places it (NUMA node of this rank's GPU, its slice of that node's
    # CPUs among the node's GPUs, bounded by the cgroup quota; pinned) unless --threads is given
    eng = h2j.Engine(local, args.threads)
    host = eng.host_info()

    # pre-built ctypes arguments: nothing but the C calls inside the timed region.  Two output
    # sets: step k + 1 is submitted before step k is waited for (the engine's asynchronous path,
    # include/h2j.h h2j_engine_submit), so one step's GPU tail and JPEG assembly overlap the next
    # step's host entropy decoding, as in a server that keeps the engine fed.
    bufs = [(ctypes.c_uint8 * len(s)).from_buffer_copy(s) for s in batch]
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    sizes = (ctypes.c_size_t * n)(*[len(s) for s in batch])
    # output capacity: 2 MiB per picture or one byte per luma pixel, whichever is larger
    cap = sum(max(2 << 20, fb // 6) for fb in frame_bytes)
    outsets = [((ctypes.c_uint8 * cap)(), (ctypes.c_size_t * n)(), (ctypes.c_size_t * n)(), (ctypes.c_int * n)())
               for _ in range(2)]

    def check(rc, status):
        if rc != 0:
            raise RuntimeError(f"transcode failed rc={rc}: {eng.error()}")
        bad = [i for i in range(n) if status[i] != 0]
        if bad:
            raise RuntimeError(f"{len(bad)} frames failed, e.g. #{bad[0]} status {status[bad[0]]}: "
                               f"{eng.frame_error(bad[0])}")

    stage_sum = {}
    chunks_all = []
    last_out = [None]  # the output set of the last step waited for (checked after the timed region)

    def collect():
        st = eng.stats()
        for k, v in st.items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        chunks_all.extend(eng.chunk_times())

    def run_steps(k_steps, record):
        if args.sync:
            for k in range(k_steps):
                out, offs, lens, status = outsets[0]
                check(eng.transcode_raw(ptrs, sizes, n, out, cap, offs, lens, status), status)
                last_out[0] = outsets[0]
                if record:
                    collect()
            return
        inflight = []
        for k in range(k_steps + 1):
            if k < k_steps:
                out, offs, lens, status = outsets[k % 2]
                inflight.append((eng.submit_raw(ptrs, sizes, n, out, cap, offs, lens, status), status))
            if k > 0:  # wait for step k - 1 (step k is parsing by now: its stats are not published yet)
                t, status = inflight.pop(0)
                check(eng.wait(t), status)
                last_out[0] = outsets[(k - 1) % 2]
                if record:
                    collect()

    def barrier():
        if dist is not None:
            dist.barrier()

    run_steps(args.warmup, False)
    barrier()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    run_steps(args.steps, True)
    t1 = time.perf_counter()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    barrier()
    elapsed = t1 - t0
    # host CPU time of this process (all threads) over the timed region, in busy cores
    host_cores = ((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / max(elapsed, 1e-9)
    elapsed, total_frames = reduce_over_ranks(dist, elapsed, n * args.steps, local)
    # outside the timed region: every JPEG of the last timed step against the oracle's md5s
    man_path = os.path.join(ROOT, "tests", "golden", "bench_manifest.json")
    manifest = json.load(open(man_path)) if os.path.exists(man_path) else {}
    out, offs, lens, _ = last_out[0]
    checked, bad, missing = verify_outputs(batch, out, offs, lens, manifest)
    bad_all = sum_over_ranks(dist, bad + missing, local)
    checked_all = sum_over_ranks(dist, checked, local)

    if rank == 0:
        steps = args.steps
        per = {k: v / steps for k, v in stage_sum.items()}
        # dominant kernel: K1 (intra prediction chain), one launch per chunk
        chunks = max(1, round(per["chunks"]))
        k1_ms = per["recon_ms"] / chunks
        frames_per_launch = n / chunks
        alg_bytes_launch = sum(frame_bytes) / chunks
        achieved = alg_bytes_launch / (k1_ms / 1e3) / 1e9
        kern_ms = (per["prep_ms"] + per["recon_ms"] + per["deblock_ms"] + per["sao_ms"] + per["jpeg_ms"]
                   + per["entropy_ms"])
        # K1's own algorithmic traffic: the int16 residual it reads (2S) + the picture it writes (b*S)
        k1_own_launch = sum(fb // (4 + bps) * (2 + bps) for fb, bps in zip(frame_bytes, frame_bps)) / chunks
        frac_k1_own = k1_own_launch / (k1_ms / 1e3) / 1e9 / HBM_PEAK_GBPS
        # BASELINE.md GPU metric: frames * B / t_kernels (K0..K5)
        frac_pipeline = sum(frame_bytes) / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBPS
        # per launch size: the full (256-picture) chunks and the tail chunks separately
        variants = {}
        fb_mean = sum(frame_bytes) / n
        for frames_c, k1c, _ in chunks_all:
            v = variants.setdefault(str(frames_c), {"launches": 0, "k1_ms": 0.0})
            v["launches"] += 1
            v["k1_ms"] += k1c
        for key, v in variants.items():
            v["avg_k1_ms"] = round(v.pop("k1_ms") / v["launches"], 4)
            v["achieved"] = round(int(key) * fb_mean / (v["avg_k1_ms"] / 1e3) / 1e9, 1)
            v["frac"] = round(v["achieved"] / HBM_PEAK_GBPS, 4)
        gpu_ms = kern_ms + per["h2d_ms"] + per["d2h_ms"]
        k1_name = {"avc1080": "h2j_k1_recon_h264", "mixed": "h2j_k1_recon_hevc+h2j_k1_recon_h264"}.get(
            args.workload, "h2j_k1_recon_hevc")
        traffic = pmc_traffic(args.workload)
        res = {
            "metric": METRIC,
            "value": total_frames / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # the sample type the decode computes in: 8-bit pictures u8, Main10 (configs[3]) u16
            "dtype": "u8" if max(frame_bps) == 1 else ("u16" if min(frame_bps) == 2 else "u8+u16"),
            "data": f"synthetic: {wl['data']} tiled to the batch",
            "config": {"workload": wl["desc"], "workload_key": args.workload,
                       "frames_per_gpu": n, "global_batch": n * world, "host_threads_per_gpu": host["threads"],
                       "host_numa_node": host["numa_node"], "host_pinned_cpus": host["pinned_cpus"],
                       "parallelism": f"independent replicas x{world}"},
            "roofline": {"bound": "hbm", "kernel": k1_name, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes_launch, "frames_per_launch": frames_per_launch,
                         "avg_launch_ms": k1_ms,
                         "frac_def": "whole-pipeline algorithmic bytes B=(4+b)S of the launch's pictures / K1 time",
                         "frac_k1_own": frac_k1_own,
                         "frac_k1_own_def": "K1's own bytes (2S residual in + b*S picture out) / K1 time",
                         "frac_pipeline": frac_pipeline,
                         "frac_pipeline_def": "BASELINE.md: frames*B / t_kernels(K0..K5)",
                         "traffic_ratio_k1_own": (traffic / k1_own_launch) if traffic else None,
                         "traffic_ratio_k1_own_def": "PMC HBM bytes per K1 launch / K1's own bytes (2S + b*S)",
                         "per_launch_size": variants},
            # value is end to end: host CABAC/CAVLC (north_star keeps entropy decoding on host
            # threads) + PCIe + K0-K5 + container.  With the job records already in HBM the
            # GPU kernels alone sustain hbm_resident_fps; gpu_pipeline_fps adds the PCIe copies.
            "timed_region": "bitstreams in host memory -> JPEG bytes in host memory (host entropy decode inside); "
                            + ("synchronous steps" if args.sync else
                               "steps pipelined two deep through h2j_engine_submit/h2j_engine_wait"),
            "hbm_resident_fps": n / (kern_ms / 1e3),
            "gpu_pipeline_fps": n / (gpu_ms / 1e3),
            "host_cpu_busy_cores": round(host_cores, 2),
            "bitstream_kb_per_frame": round(sum(len(b) for b in batch) / n / 1024, 1),
            "parse_us_per_kb_wall": round(per["parse_run_ms"] * 1e3 / (sum(len(b) for b in batch) / 1024), 3),
            "parse_core_us_per_kb": parse_core_us_per_kb(per, host["threads"], batch),
            "parse_core_def": "pool wall time from the batch's first to its last parsed picture x host threads / KB "
                              "(r02 used submission -> last parsed, which counted the wait behind the previous batch)",
            "stages_ms_per_step": {k: round(v, 3) for k, v in per.items() if k.endswith("_ms")},
            # the JPEG payload copy's own rate (PCIe, pinned host buffer)
            "d2h_payload_MB_per_step": round(per.get("payload_bytes", 0.0) / 1e6, 2),
            "d2h_payload_copied_MB_per_step": round(per.get("payload_copied_bytes", 0.0) / 1e6, 2),
            "d2h_payload_GBps": round(per.get("payload_copied_bytes", 0.0) / max(per.get("d2h_payload_ms", 0.0), 1e-9) / 1e6, 2),
            "h2d_MB_per_step": round(per.get("h2d_bytes", 0.0) / 1e6, 2),
            "h2d_GBps": round(per.get("h2d_bytes", 0.0) / max(per.get("h2d_ms", 0.0), 1e-9) / 1e6, 2),
            "outputs_verified": bool(manifest) and bad_all == 0,
            "outputs_checked": {"pictures": checked_all, "mismatched_or_unknown": bad_all,
                                "def": "md5 of every JPEG of the last timed step (all ranks) == md5 of the oracle's "
                                       "JPEG of its stream (tests/golden/bench_manifest.json, "
                                       "tools/make_bench_manifest.py); checked after the timed region"},
        }
        # configs[0]-style single calls: the reference fixture and one stream of this workload
        if not args.no_single_call:
            with open(os.path.join(ROOT, "tests", "golden", "img01.h265"), "rb") as fx:
                fixture = fx.read()
            res["single_call_ms"] = single_call_latency([("img01.h265", fixture), ("workload_stream0", streams[0])])
        # N = 1 only: configs[1] on the SURVEY.md §8(d)-aim set (100-250 KB per picture), and the
        # end-to-end rate against the host entropy threads on this one GPU (DESIGN.md §7 predicts
        # the 1 -> 8 GPU curve from it)
        if world == 1 and args.workload in ("hevc1080", "avc1080") and not args.no_aim:
            # hevc1080: `value` is already the §8(d)-aim set; the lighter round 1-5 set is value_light.
            # avc1080: value_aim = configs[2] on the 100-250 KB/picture set
            key, hkey = ("value_light", "hevc1080_light") if args.workload == "hevc1080" else ("value_aim", "avc1080_heavy")
            heavy = load_streams(WORKLOADS[hkey]["streams"])
            hbatch = [heavy[i % len(heavy)] for i in range(n)]
            fps, hper = timed_batches(eng, hbatch, 4, 1)
            res[key] = fps
            res[key + "_def"] = (f"{'configs[1]' if args.workload == 'hevc1080' else 'configs[2]'} on "
                                 f"{WORKLOADS[hkey]['streams'].rsplit('/', 1)[0]} ({len(heavy)} generator 1080p streams, "
                                 f"{sum(len(b) for b in hbatch) / n / 1024:.1f} KB/picture), same engine and timing")
            res[key + "_parse_core_us_per_kb"] = parse_core_us_per_kb(hper, host["threads"], hbatch)
            # the dominant kernel on that set too (same definitions as `roofline`)
            hch = max(1, round(hper.get("chunks", 1)))
            hk1 = hper["recon_ms"] / hch
            hach = alg_bytes_per_frame(WORKLOADS[hkey]) * n / hch / (hk1 / 1e3) / 1e9
            res[key + "_roofline"] = {"kernel": k1_name, "avg_launch_ms": hk1, "frames_per_launch": n / hch,
                                      "achieved": hach, "frac": hach / HBM_PEAK_GBPS,
                                      "hbm_resident_fps": n / ((hper["prep_ms"] + hper["recon_ms"] + hper["deblock_ms"] +
                                                                hper["sao_ms"] + hper["jpeg_ms"] + hper["entropy_ms"]) / 1e3)}
            sweep = {}
            for t in (2, 4, 8, 16):
                if t > host["threads"]:
                    continue
                e2 = eng if t == host["threads"] else h2j.Engine(local, t)
                fps_t, _ = timed_batches(e2, batch, 2 if t >= 8 else 1, 1)
                sweep[str(t)] = round(fps_t, 1)
                if e2 is not eng:
                    e2.close()
            res["host_thread_sweep_fps"] = sweep
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(streams, host["threads"])
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
