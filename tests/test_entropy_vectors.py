"""CPU: the high-entropy vectors (tests/golden/entropy, tools/make_streams.py entropy) really
drive K5d's global-memory emission path next to LDS-path tiles: from the oracle's
JPEG, the payload bits of every 256-block tile (K5's tile, blocks in MCU order Y0..Y3 Cb Cr) are
recomputed with the JPEG's own Huffman code lengths; some tile must span more than kEmitWords
(2048) 32-bit words and some tile fewer.  tests/test_gpu_hevc.py checks the GPU's JPEG on both
paths byte for byte."""
import glob
import os
import struct

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read

K_TILE = 256
K_EMIT_WORDS = 2048
PATHS = sorted(glob.glob(os.path.join(golden("entropy"), "*.h265")))


def huffman_lengths(jpg):
    """{(class, id): {symbol: code length}} from the DHT segments"""
    out = {}
    i = 2
    while i < len(jpg) - 4:
        if jpg[i] != 0xFF:
            i += 1
            continue
        m = jpg[i + 1]
        if m == 0xDA:
            break
        seg_len = struct.unpack(">H", jpg[i + 2:i + 4])[0]
        if m == 0xC4:
            p = i + 4
            end = i + 2 + seg_len
            while p < end:
                tc, th = jpg[p] >> 4, jpg[p] & 15
                counts = jpg[p + 1:p + 17]
                syms = jpg[p + 17:p + 17 + sum(counts)]
                lens, k = {}, 0
                for L, c in enumerate(counts, start=1):
                    for _ in range(c):
                        lens[syms[k]] = L
                        k += 1
                out[(tc, th)] = lens
                p += 17 + sum(counts)
        i += 2 + seg_len
    return out


def nbits(v):
    return int(abs(int(v))).bit_length()




@pytest.mark.parametrize("path", PATHS, ids=[os.path.basename(p) for p in PATHS])
def test_entropy_vectors_straddle_the_lds_limit(path):
    jpg = O.transcode(read(path))
    lens = huffman_lengths(jpg)
    w, h, _, coefs = O.jpeg_parse(jpg)
    pred = [128, 128, 128]  # FFmpeg mjpeg: last_dc starts at 128 << intra_dc_precision
    bits = []
    for mcu in coefs:
        for b in range(6):
            comp = 0 if b < 4 else b - 3
            tab = 0 if comp == 0 else 1
            blk = mcu[b]
            diff = int(blk[0]) - pred[comp]
            pred[comp] = int(blk[0])
            cat = nbits(diff)
            n = lens[(0, tab)][cat] + cat
            run = 0
            nz = np.nonzero(blk[1:])[0]
            last = nz[-1] + 1 if len(nz) else 0
            for k in range(1, last + 1):
                v = int(blk[k])
                if v == 0:
                    run += 1
                    continue
                while run >= 16:
                    n += lens[(1, tab)][0xF0]
                    run -= 16
                s = nbits(v)
                n += lens[(1, tab)][(run << 4) | s] + s
                run = 0
            if last < 63:
                n += lens[(1, tab)][0x00]
            bits.append(n)
    bits = np.array(bits)
    words = [(int(bits[t:t + K_TILE].sum()) + 31) // 32 + 1 for t in range(0, len(bits), K_TILE)]
    assert max(words) > K_EMIT_WORDS, words
    assert min(words) <= K_EMIT_WORDS, words
