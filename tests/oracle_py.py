"""ctypes access to the ORACLE (oracle/liboracle.so) — test infrastructure only.

The oracle is the CPU restatement of the reference's arithmetic (see
oracle/oracle.h).  Tests use it as the checker; the product never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SO = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


class OraclePicture(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("bit_depth", ctypes.c_int),
                ("chroma_format", ctypes.c_int), ("planes", ctypes.POINTER(ctypes.c_uint16) * 3),
                ("stride", ctypes.c_int * 3)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        l = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        l.oracle_hevc_decode.argtypes = [u8p, ctypes.c_long, ctypes.c_int, ctypes.POINTER(OraclePicture)]
        l.oracle_h264_decode.argtypes = [u8p, ctypes.c_long, ctypes.c_int, ctypes.POINTER(OraclePicture)]
        l.oracle_free_picture.argtypes = [ctypes.POINTER(OraclePicture)]
        l.oracle_transcode.restype = ctypes.c_long
        l.oracle_transcode.argtypes = [u8p, ctypes.c_long, ctypes.c_char_p, u8p, ctypes.c_long]
        l.oracle_jpeg_parse.argtypes = [u8p, ctypes.c_long, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                        u8p, ctypes.POINTER(ctypes.c_int16), ctypes.c_int]
        l.oracle_jpeg_from_coeffs.restype = ctypes.c_long
        l.oracle_jpeg_from_coeffs.argtypes = [ctypes.POINTER(ctypes.c_int16), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_char_p, u8p, ctypes.c_long]
        l.oracle_jpeg_coeffs.argtypes = [u8p, u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int16), ctypes.POINTER(ctypes.c_int)]
        l.oracle_jpeg_encode.restype = ctypes.c_long
        l.oracle_jpeg_encode.argtypes = [u8p, u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_char_p, u8p, ctypes.c_long]
        l.oracle_fdct.argtypes = [ctypes.POINTER(ctypes.c_int16)]
        _lib = l
    return _lib


def _buf(b: bytes):
    return (ctypes.c_uint8 * len(b)).from_buffer_copy(b)


def decode(stream: bytes, codec: int = 265, skip_loop_filter: bool = False):
    """-> (Y, U, V) uint16 arrays + bit depth, or raises."""
    pic = OraclePicture()
    fn = lib().oracle_hevc_decode if codec == 265 else lib().oracle_h264_decode
    r = fn(_buf(stream), len(stream), 1 if skip_loop_filter else 0, ctypes.byref(pic))
    if r != 0:
        raise RuntimeError(f"oracle decode failed {r}")
    w, h = pic.width, pic.height
    planes = []
    for c in range(3):
        cw, ch = (w, h) if c == 0 else (w // 2, h // 2)
        arr = np.ctypeslib.as_array(pic.planes[c], shape=(ch * pic.stride[c],)).copy()
        planes.append(arr.reshape(ch, pic.stride[c])[:, :cw].copy())
    bd = pic.bit_depth
    lib().oracle_free_picture(ctypes.byref(pic))
    return planes[0], planes[1], planes[2], bd


def transcode(stream: bytes, com: bytes = b"Lavc58.117.101") -> bytes:
    cap = len(stream) * 4 + (16 << 20)
    out = (ctypes.c_uint8 * cap)()
    n = lib().oracle_transcode(_buf(stream), len(stream), com, out, cap)
    if n <= 0:
        raise RuntimeError(f"oracle transcode failed {n}")
    return bytes(out[:n])


def jpeg_parse(jpg: bytes):
    w = ctypes.c_int()
    h = ctypes.c_int()
    dqt = (ctypes.c_uint8 * 64)()
    n = lib().oracle_jpeg_parse(_buf(jpg), len(jpg), ctypes.byref(w), ctypes.byref(h), dqt, None, 0)
    coefs = np.zeros(n * 384, dtype=np.int16)
    n2 = lib().oracle_jpeg_parse(_buf(jpg), len(jpg), ctypes.byref(w), ctypes.byref(h), dqt,
                                 coefs.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), n)
    if n2 != n:
        raise RuntimeError(f"jpeg parse failed {n2}")
    return w.value, h.value, bytes(dqt), coefs.reshape(n, 6, 64)


def jpeg_from_coeffs(coefs: np.ndarray, w: int, h: int, qscale: int, com: bytes) -> bytes:
    c = np.ascontiguousarray(coefs, dtype=np.int16)
    cap = c.size * 4 + 65536
    out = (ctypes.c_uint8 * cap)()
    n = lib().oracle_jpeg_from_coeffs(c.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), w, h, qscale, com, out, cap)
    if n <= 0:
        raise RuntimeError("jpeg emission failed")
    return bytes(out[:n])


def to8(plane: np.ndarray, bd: int) -> np.ndarray:
    if bd == 8:
        return plane.astype(np.uint8)
    v = (plane.astype(np.int32) + (1 << (bd - 9))) >> (bd - 8)
    return np.minimum(v, 255).astype(np.uint8)


def jpeg_coeffs(y, u, v):
    """Quantised zigzag coefficients [nmcu,6,64] + qscale for 8-bit planes."""
    h, w = y.shape
    y = np.ascontiguousarray(y, dtype=np.uint8)
    u = np.ascontiguousarray(u, dtype=np.uint8)
    v = np.ascontiguousarray(v, dtype=np.uint8)
    nmcu = ((w + 15) // 16) * ((h + 15) // 16)
    out = np.zeros(nmcu * 384, dtype=np.int16)
    qs = ctypes.c_int()
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    lib().oracle_jpeg_coeffs(p(y), p(u), p(v), w, h, w, w // 2,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), ctypes.byref(qs))
    return qs.value, out.reshape(nmcu, 6, 64)
