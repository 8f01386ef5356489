"""Python binding of libH265ToJpeg.so (ctypes over the C ABI in include/h2j.h).

This mirrors the reference's operator surface for the path:
``IDecoder::getInstance()->H265ToJpeg(in, out)`` (/root/reference/export_inc/IDecoder.h:29,35)
is :func:`h265_to_jpeg`; the batch engine underneath it is :class:`Engine`.
There is no CPU fallback: constructing an :class:`Engine` without a HIP
device raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_NAME = "libH265ToJpeg.so"
_lib = None


def lib_path() -> str:
    # H2J_LIB_DIR selects an alternative build of the same libraries (e.g. build/prof)
    return os.path.join(os.environ.get("H2J_LIB_DIR", _HERE), _LIB_NAME)


def load_library() -> ctypes.CDLL:
    """Load libH265ToJpeg.so (and, through its RUNPATH, libh2j_hip.so)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run `make -C h264-h265-to-jpeg_amd` or __graft_entry__.build()")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    szp = ctypes.POINTER(ctypes.c_size_t)
    lib.h2j_engine_create.restype = ctypes.c_void_p
    lib.h2j_engine_create.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.h2j_engine_destroy.argtypes = [ctypes.c_void_p]
    lib.h2j_engine_error.restype = ctypes.c_char_p
    lib.h2j_engine_error.argtypes = [ctypes.c_void_p]
    lib.h2j_engine_transcode.restype = ctypes.c_int
    lib.h2j_engine_transcode.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(u8p), szp, u8p,
                                         ctypes.c_size_t, szp, szp, ctypes.POINTER(ctypes.c_int)]
    lib.h2j_engine_decode.restype = ctypes.c_int
    lib.h2j_engine_decode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_uint16), ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
    lib.h2j_engine_decode_batch.restype = ctypes.c_int
    lib.h2j_engine_decode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(u8p), szp, ctypes.c_int,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_uint16), ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_int)]
    lib.h2j_engine_jpeg_coeffs.restype = ctypes.c_int
    lib.h2j_engine_jpeg_coeffs.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int16),
                                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
    lib.h2j_engine_submit.restype = ctypes.c_int64
    lib.h2j_engine_submit.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(u8p), szp, u8p,
                                      ctypes.c_size_t, szp, szp, ctypes.POINTER(ctypes.c_int)]
    lib.h2j_engine_wait.restype = ctypes.c_int
    lib.h2j_engine_wait.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.h2j_engine_stats.restype = ctypes.c_int
    lib.h2j_engine_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    lib.h2j_engine_frame_error.restype = ctypes.c_char_p
    lib.h2j_engine_frame_error.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.h2j_engine_host_info.restype = ctypes.c_int
    lib.h2j_engine_host_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.h2j_device_count.restype = ctypes.c_int
    lib.h2j_engine_chunk_times.restype = ctypes.c_int
    lib.h2j_engine_chunk_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    lib.h2j_version.restype = ctypes.c_char_p
    lib.h2j_gpu_device_count.restype = ctypes.c_int
    _lib = lib
    return lib


def device_count() -> int:
    return int(load_library().h2j_gpu_device_count())


def _u8(buf: bytes):
    arr = (ctypes.c_uint8 * len(buf)).from_buffer_copy(buf)
    return arr


STAT_KEYS = ["parse_ms", "h2d_ms", "recon_ms", "deblock_ms", "sao_ms", "jpeg_ms", "d2h_ms",
             "assemble_ms", "total_ms", "frames", "alg_bytes", "entropy_ms", "prep_ms", "chunks", "pack_ms",
             "parse_run_ms", "d2h_stats_ms", "d2h_payload_ms", "payload_bytes", "host_grow_ms", "h2d_bytes",
             "payload_copied_bytes"]


class Engine:
    """One process-per-GPU transcoding engine (host entropy threads + HIP pipeline)."""

    def __init__(self, device: int = 0, host_threads: int = 0):
        self._lib = load_library()
        self._h = self._lib.h2j_engine_create(int(device), int(host_threads))
        if not self._h:
            raise RuntimeError("h2j_engine_create failed: no usable HIP device for the MI355X pipeline")

    def close(self) -> None:
        if self._h:
            self._lib.h2j_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        return self._lib.h2j_engine_error(self._h).decode(errors="replace")

    def frame_error(self, i: int) -> str:
        """Message of picture i of the last transcode ('' if it succeeded)."""
        return self._lib.h2j_engine_frame_error(self._h, int(i)).decode(errors="replace")

    def host_info(self) -> dict:
        """Host entropy pool placement (include/h2j.h h2j_engine_host_info)."""
        arr = (ctypes.c_int * 4)()
        self._lib.h2j_engine_host_info(self._h, arr, 4)
        return {"threads": arr[0], "numa_node": arr[1], "pinned_cpus": arr[2], "first_cpu": arr[3]}

    def transcode(self, streams: Sequence[bytes]) -> List[Optional[bytes]]:
        """Annex-B H.264/H.265 stills -> JPEG bytes (None for items that failed)."""
        n = len(streams)
        if n == 0:
            return []
        bufs = [_u8(s) for s in streams]
        ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
        sizes = (ctypes.c_size_t * n)(*[len(s) for s in streams])
        # JPEG bytes: usually well under 1 MiB per still; on -50 (output buffer too small) retry larger
        cap = sum(max(1 << 20, 4 * len(s)) for s in streams)
        offs = (ctypes.c_size_t * n)()
        lens = (ctypes.c_size_t * n)()
        status = (ctypes.c_int * n)()
        for _ in range(4):
            out = (ctypes.c_uint8 * cap)()
            rc = self._lib.h2j_engine_transcode(self._h, n, ptrs, sizes, out, cap, offs, lens, status)
            if not any(status[i] == -50 for i in range(n)):
                break
            cap *= 4
        if rc < 0 and rc != -3:
            raise RuntimeError(f"h2j_engine_transcode failed ({rc}): {self.error()}")
        mv = memoryview(out)
        return [bytes(mv[offs[i]:offs[i] + lens[i]]) if status[i] == 0 else None for i in range(n)]

    def transcode_raw(self, ptrs, sizes, n, out, cap, offs, lens, status) -> int:
        """Zero-copy variant for benchmarks (pre-built ctypes arrays)."""
        return self._lib.h2j_engine_transcode(self._h, n, ptrs, sizes, out, cap, offs, lens, status)

    def submit_raw(self, ptrs, sizes, n, out, cap, offs, lens, status) -> int:
        """Asynchronous batch (h2j_engine_submit): returns a ticket; the ctypes arrays must stay
        alive until wait(ticket)."""
        t = self._lib.h2j_engine_submit(self._h, n, ptrs, sizes, out, cap, offs, lens, status)
        if t <= 0:
            raise RuntimeError(f"h2j_engine_submit failed ({t})")
        return t

    def wait(self, ticket: int) -> int:
        return self._lib.h2j_engine_wait(self._h, int(ticket))

    def transcode_async(self, batches: Sequence[Sequence[bytes]]) -> List[List[Optional[bytes]]]:
        """Several batches through the asynchronous path, all submitted before the first wait."""
        held, tickets = [], []
        for streams in batches:
            n = len(streams)
            bufs = [_u8(s) for s in streams]
            ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
            sizes = (ctypes.c_size_t * n)(*[len(s) for s in streams])
            cap = sum(max(2 << 20, 4 * len(s)) for s in streams)
            out = (ctypes.c_uint8 * cap)()
            offs, lens, status = (ctypes.c_size_t * n)(), (ctypes.c_size_t * n)(), (ctypes.c_int * n)()
            held.append((bufs, ptrs, sizes, out, offs, lens, status, n))
            tickets.append(self.submit_raw(ptrs, sizes, n, out, cap, offs, lens, status))
        res = []
        for t, (bufs, ptrs, sizes, out, offs, lens, status, n) in zip(tickets, held):
            rc = self.wait(t)
            if rc < 0 and rc != -3:
                raise RuntimeError(f"h2j_engine_wait failed ({rc}): {self.error()}")
            mv = memoryview(out)
            res.append([bytes(mv[offs[i]:offs[i] + lens[i]]) if status[i] == 0 else None for i in range(n)])
        return res

    def decode(self, stream: bytes, stage: int = 0):
        """Decoded picture planes (uint16 numpy Y, U, V) of the first picture.

        stage 0: final, 1: before loop filters, 2: after deblocking (before SAO).
        """
        buf = _u8(stream)
        cap = 8192 * 8192 * 3 // 2
        out = np.zeros(cap, dtype=np.uint16)
        info = (ctypes.c_int * 3)()
        rc = self._lib.h2j_engine_decode(self._h, buf, len(stream), int(stage),
                                         out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), cap, info)
        if rc < 0:
            raise RuntimeError(f"h2j_engine_decode failed ({rc}): {self.error()}")
        return self._planes(out, info)

    def decode_batch(self, streams: Sequence[bytes], pick: int, stage: int = 0):
        """Planes of picture `pick` of `streams` reconstructed as one GPU batch (the launch shapes
        of a production chunk of that many pictures)."""
        n = len(streams)
        bufs = [_u8(s) for s in streams]
        ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
        sizes = (ctypes.c_size_t * n)(*[len(s) for s in streams])
        cap = 8192 * 8192 * 3 // 2
        out = np.zeros(cap, dtype=np.uint16)
        info = (ctypes.c_int * 3)()
        rc = self._lib.h2j_engine_decode_batch(self._h, n, ptrs, sizes, int(stage), int(pick),
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), cap, info)
        if rc < 0:
            raise RuntimeError(f"h2j_engine_decode_batch failed ({rc}): {self.error()}")
        return self._planes(out, info)

    @staticmethod
    def _planes(out, info):
        w, h, bd = info[0], info[1], info[2]
        ys = w * h
        cs = (w // 2) * (h // 2)
        y = out[:ys].reshape(h, w).copy()
        u = out[ys:ys + cs].reshape(h // 2, w // 2).copy()
        v = out[ys + cs:ys + 2 * cs].reshape(h // 2, w // 2).copy()
        return y, u, v, bd

    def jpeg_coeffs(self, stream: bytes):
        """(qscale, int16 array [nmcu, 6, 64]) computed by the GPU JPEG stage."""
        buf = _u8(stream)
        cap = (8192 // 16) * (8192 // 16) * 384
        out = np.zeros(cap, dtype=np.int16)
        info = (ctypes.c_int * 4)()
        rc = self._lib.h2j_engine_jpeg_coeffs(self._h, buf, len(stream),
                                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), cap, info)
        if rc < 0:
            raise RuntimeError(f"h2j_engine_jpeg_coeffs failed ({rc}): {self.error()}")
        nmcu = info[3]
        return info[2], out[:nmcu * 384].reshape(nmcu, 6, 64).copy()

    def chunk_times(self) -> list:
        """[(pictures, K1 ms, K0..K5 ms)] per chunk of the last transcode."""
        cap = 4096
        arr = (ctypes.c_double * (3 * cap))()
        n = self._lib.h2j_engine_chunk_times(self._h, arr, cap)
        return [(int(arr[3 * i]), arr[3 * i + 1], arr[3 * i + 2]) for i in range(min(n, cap))]

    def stats(self) -> dict:
        arr = (ctypes.c_double * len(STAT_KEYS))()
        self._lib.h2j_engine_stats(self._h, arr, len(STAT_KEYS))
        return {k: arr[i] for i, k in enumerate(STAT_KEYS)}


def h265_to_jpeg(input_path: str, output_path: str) -> bool:
    """Python mirror of IDecoder::getInstance()->H265ToJpeg(in, out)."""
    if not input_path or not output_path:
        return False
    try:
        with open(input_path, "rb") as f:
            data = f.read()
    except OSError:
        return False
    eng = _shared_engine()
    out = eng.transcode([data])[0]
    if out is None:
        return False
    try:
        with open(output_path, "wb+") as f:
            f.write(out)
    except OSError:
        return False
    return True


_ENGINE: Optional[Engine] = None


def _shared_engine() -> Engine:
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine()
    return _ENGINE
