"""Generate the H.264 CAVLC VLC tables (ITU-T H.264 Tables 9-5, 9-7, 9-8,
9-9(a), 9-10 and the intra column of Table 9-4) as C headers for the host
parser and tools/h264gen (the oracle has an independent hand-typed copy,
oracle/cavlc_spec.h), after checking every table is prefix-free
(and printing its Kraft sum).  Spec data, written once here.

  python tools/gen_cavlc_tables.py
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# coeff_token: (TrailingOnes, TotalCoeff) -> codes for nC ranges
# [0 <= nC < 2, 2 <= nC < 4, 4 <= nC < 8, nC == -1 (4:2:0 chroma DC)];
# 8 <= nC is a 6-bit FLC handled in code.
COEFF_TOKEN = {
    (0, 0): ("1", "11", "1111", "01"),
    (0, 1): ("000101", "001011", "001111", "000111"),
    (1, 1): ("01", "10", "1110", "1"),
    (0, 2): ("00000111", "000111", "001011", "000100"),
    (1, 2): ("000100", "00111", "01111", "000110"),
    (2, 2): ("001", "011", "1101", "001"),
    (0, 3): ("000000111", "0000111", "001000", "000011"),
    (1, 3): ("00000110", "001010", "01100", "0000011"),
    (2, 3): ("0000101", "001001", "01110", "0000010"),
    (3, 3): ("00011", "0101", "1100", "000101"),
    (0, 4): ("0000000111", "00000111", "0001111", "000010"),
    (1, 4): ("000000110", "000110", "01010", "00000011"),
    (2, 4): ("00000101", "000101", "01011", "00000010"),
    (3, 4): ("000011", "0100", "1011", "0000000"),
    (0, 5): ("00000000111", "00000100", "0001011", None),
    (1, 5): ("0000000110", "0000110", "01000", None),
    (2, 5): ("000000101", "0000101", "01001", None),
    (3, 5): ("0000100", "00110", "1010", None),
    (0, 6): ("0000000001111", "000000111", "0001001", None),
    (1, 6): ("00000000110", "00000110", "001110", None),
    (2, 6): ("0000000101", "00000101", "001101", None),
    (3, 6): ("00000100", "001000", "1001", None),
    (0, 7): ("0000000001011", "00000001111", "0001000", None),
    (1, 7): ("0000000001110", "000000110", "001010", None),
    (2, 7): ("00000000101", "000000101", "001001", None),
    (3, 7): ("000000100", "000100", "1000", None),
    (0, 8): ("0000000001000", "00000001011", "00001111", None),
    (1, 8): ("0000000001010", "00000001110", "0001110", None),
    (2, 8): ("0000000001101", "00000001101", "0001101", None),
    (3, 8): ("0000000100", "0000100", "01101", None),
    (0, 9): ("00000000001111", "000000001111", "00001011", None),
    (1, 9): ("00000000001110", "00000001010", "00001110", None),
    (2, 9): ("0000000001001", "00000001001", "0001010", None),
    (3, 9): ("00000000100", "000000100", "001100", None),
    (0, 10): ("00000000001011", "000000001011", "000001111", None),
    (1, 10): ("00000000001010", "000000001110", "00001010", None),
    (2, 10): ("00000000001101", "000000001101", "00001101", None),
    (3, 10): ("0000000001100", "00000001100", "0001100", None),
    (0, 11): ("000000000001111", "000000001000", "000001011", None),
    (1, 11): ("000000000001110", "000000001010", "000001110", None),
    (2, 11): ("00000000001001", "000000001001", "00001001", None),
    (3, 11): ("00000000001100", "00000001000", "00001100", None),
    (0, 12): ("000000000001011", "0000000001111", "000001000", None),
    (1, 12): ("000000000001010", "0000000001110", "000001010", None),
    (2, 12): ("000000000001101", "0000000001101", "000001101", None),
    (3, 12): ("00000000001000", "000000001100", "00001000", None),
    (0, 13): ("0000000000001111", "0000000001011", "0000001101", None),
    (1, 13): ("000000000000001", "0000000001010", "000000111", None),
    (2, 13): ("000000000001001", "0000000001001", "000001001", None),
    (3, 13): ("000000000001100", "0000000001100", "000001100", None),
    (0, 14): ("0000000000001011", "0000000000111", "0000001001", None),
    (1, 14): ("0000000000001110", "00000000001011", "0000001100", None),
    (2, 14): ("0000000000001101", "0000000000110", "0000001011", None),
    (3, 14): ("000000000001000", "0000000001000", "0000001010", None),
    (0, 15): ("0000000000000111", "00000000001001", "0000000101", None),
    (1, 15): ("0000000000001010", "00000000001000", "0000001000", None),
    (2, 15): ("0000000000001001", "00000000001010", "0000000111", None),
    (3, 15): ("0000000000001100", "0000000000001", "0000000110", None),
    (0, 16): ("0000000000000100", "00000000000111", "0000000001", None),
    (1, 16): ("0000000000000110", "00000000000110", "0000000100", None),
    (2, 16): ("0000000000000101", "00000000000101", "0000000011", None),
    (3, 16): ("0000000000001000", "00000000000100", "0000000010", None),
}

# total_zeros for 4x4 blocks, tzVlcIndex = TotalCoeff 1..15 (Tables 9-7, 9-8)
TOTAL_ZEROS = {
    1: "1 011 010 0011 0010 00011 00010 000011 000010 0000011 0000010 00000011 00000010 000000011 000000010 000000001",
    2: "111 110 101 100 011 0101 0100 0011 0010 00011 00010 000011 000010 000001 000000",
    3: "0101 111 110 101 0100 0011 100 011 0010 00011 00010 000001 00001 000000",
    4: "00011 111 0101 0100 110 101 100 0011 011 0010 00010 00001 00000",
    5: "0101 0100 0011 111 110 101 100 011 0010 00001 0001 00000",
    6: "000001 00001 111 110 101 100 011 010 0001 001 000000",
    7: "000001 00001 101 100 011 11 010 0001 001 000000",
    8: "000001 0001 00001 011 11 10 010 001 000000",
    9: "000001 000000 0001 11 10 001 01 00001",
    10: "00001 00000 001 11 10 01 0001",
    11: "0000 0001 001 010 1 011",
    12: "0000 0001 01 1 001",
    13: "000 001 1 01",
    14: "00 01 1",
    15: "0 1",
}
# total_zeros for 4:2:0 chroma DC, tzVlcIndex 1..3 (Table 9-9a)
TOTAL_ZEROS_DC = {1: "1 01 001 000", 2: "1 01 00", 3: "1 0"}
# run_before, zerosLeft 1..6 and > 6 (Table 9-10)
RUN_BEFORE = {
    1: "1 0",
    2: "1 01 00",
    3: "11 10 01 00",
    4: "11 10 01 001 000",
    5: "11 10 011 010 001 000",
    6: "11 000 001 011 010 101 100",
    7: "111 110 101 100 011 010 001 0001 00001 000001 0000001 00000001 000000001 0000000001 00000000001",
}
# Table 9-4, chroma_format_idc 1/2, Intra_4x4 / Intra_8x8 column: codeNum -> coded_block_pattern
CBP_INTRA = [47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19, 21, 26, 28, 35,
             37, 42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34, 36, 40, 38, 41]


def check(name, codes):
    codes = [c for c in codes if c]
    for a in codes:
        for b in codes:
            if a is not b and b.startswith(a):
                raise SystemExit(f"{name}: {a} is a prefix of {b}")
    kraft = sum(2.0 ** -len(c) for c in codes)
    if kraft > 1.0 + 1e-12:
        raise SystemExit(f"{name}: Kraft sum {kraft} > 1")
    return kraft


def main():
    for col, nm in enumerate(["nC0", "nC2", "nC4", "nCm1"]):
        k = check(f"coeff_token {nm}", [v[col] for v in COEFF_TOKEN.values()])
        print(f"coeff_token {nm}: {sum(1 for v in COEFF_TOKEN.values() if v[col])} codes, Kraft {k:.6f}")
    for t, s in TOTAL_ZEROS.items():
        codes = s.split()
        assert len(codes) == 17 - t, (t, len(codes))
        print(f"total_zeros tzVlcIndex {t}: Kraft {check(f'tz{t}', codes):.6f}")
    for t, s in TOTAL_ZEROS_DC.items():
        assert len(s.split()) == 5 - t
        check(f"tzdc{t}", s.split())
    for z, s in RUN_BEFORE.items():
        check(f"rb{z}", s.split())
    assert sorted(CBP_INTRA) == list(range(48))

    # C tables: code bits + lengths
    ct = []  # [4][4][17] (len, code)
    for col in range(4):
        rows = []
        for t1 in range(4):
            ent = []
            for tc in range(17):
                c = COEFF_TOKEN.get((t1, tc))
                c = c[col] if c else None
                ent.append((len(c), int(c, 2)) if c else (0, 0))
            rows.append(ent)
        ct.append(rows)
    out = ["/* Generated by tools/gen_cavlc_tables.py: H.264 CAVLC VLC tables (spec data). */",
           "#ifndef H2J_CAVLC_TABLES_H", "#define H2J_CAVLC_TABLES_H", "#include <stdint.h>", "",
           "/* coeff_token [nC class: 0 (0..1), 1 (2..3), 2 (4..7), 3 (-1 chroma DC)][TrailingOnes][TotalCoeff] */",
           "static const uint8_t kCoeffTokenLen[4][4][17] = {"]
    for col in range(4):
        out.append("    {" + ", ".join("{" + ", ".join(str(e[0]) for e in ct[col][t1]) + "}" for t1 in range(4)) + "},")
    out.append("};")
    out.append("static const uint16_t kCoeffTokenCode[4][4][17] = {")
    for col in range(4):
        out.append("    {" + ", ".join("{" + ", ".join(str(e[1]) for e in ct[col][t1]) + "}" for t1 in range(4)) + "},")
    out.append("};")
    out.append("/* total_zeros [tzVlcIndex 1..15 -> 0..14][total_zeros 0..15] */")
    tl = [[0] * 16 for _ in range(15)]
    tcodes = [[0] * 16 for _ in range(15)]
    for t, s in TOTAL_ZEROS.items():
        for z, c in enumerate(s.split()):
            tl[t - 1][z] = len(c)
            tcodes[t - 1][z] = int(c, 2)
    out.append("static const uint8_t kTotalZerosLen[15][16] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in tl) + "};")
    out.append("static const uint8_t kTotalZerosCode[15][16] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in tcodes) + "};")
    dl = [[0] * 4 for _ in range(3)]
    dc = [[0] * 4 for _ in range(3)]
    for t, s in TOTAL_ZEROS_DC.items():
        for z, c in enumerate(s.split()):
            dl[t - 1][z] = len(c)
            dc[t - 1][z] = int(c, 2)
    out.append("/* total_zeros, 4:2:0 chroma DC [tzVlcIndex 1..3 -> 0..2][total_zeros 0..3] */")
    out.append("static const uint8_t kTotalZerosDcLen[3][4] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in dl) + "};")
    out.append("static const uint8_t kTotalZerosDcCode[3][4] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in dc) + "};")
    rl = [[0] * 15 for _ in range(7)]
    rc = [[0] * 15 for _ in range(7)]
    for z, s in RUN_BEFORE.items():
        for r, c in enumerate(s.split()):
            rl[z - 1][r] = len(c)
            rc[z - 1][r] = int(c, 2)
    out.append("/* run_before [min(zerosLeft, 7) - 1][run_before] */")
    out.append("static const uint8_t kRunBeforeLen[7][15] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in rl) + "};")
    out.append("static const uint16_t kRunBeforeCode[7][15] = {" + ", ".join("{" + ", ".join(map(str, r)) + "}" for r in rc) + "};")
    out.append("/* coded_block_pattern me(v), Intra_4x4 / Intra_8x8, chroma_format_idc 1 */")
    out.append("static const uint8_t kCbpIntra[48] = {" + ", ".join(map(str, CBP_INTRA)) + "};")
    out += ["", "#endif", ""]
    text = "\n".join(out)
    # the oracle keeps its own hand-typed copy (oracle/cavlc_spec.h), checked against these by
    # tests/test_cavlc_tables.py
    for path in ("h264-h265-to-jpeg_amd/csrc/host/cavlc_tables.h", "tools/h264gen/cavlc_tables.h"):
        open(os.path.join(ROOT, path), "w").write(text)
        print("wrote", path)


if __name__ == "__main__":
    main()
