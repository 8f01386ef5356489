"""Annex-B wire-format variants of a stream that must transcode to the same
JPEG as the original: access-unit delimiters, SEI, a second
picture (only picture 0 is used, /root/reference/src/Decoder.cpp:342-355),
trailing_zero_8bits, 3-byte start codes."""

SC4 = b"\x00\x00\x00\x01"


def split_nals(s):
    """(start, end) of each NAL payload (header onward) in an Annex-B stream."""
    out, i, n = [], 0, len(s)
    starts = []
    while i + 3 <= n:
        if s[i] == 0 and s[i + 1] == 0 and s[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    for k, st in enumerate(starts):
        en = starts[k + 1] - 3 if k + 1 < len(starts) else n
        while en > st and s[en - 1] == 0:
            en -= 1
        out.append(s[st:en])
    return out


def join(nals, sc=SC4):
    return b"".join(sc + x for x in nals)


def aud(codec):
    return b"\x09\x10" if codec == 264 else b"\x46\x01\x10"


def sei(codec):
    # user_data_unregistered (payloadType 5), 17 bytes: 16-byte UUID + 1 byte
    body = bytes([5, 17]) + bytes(range(0x10, 0x20)) + b"\x2a" + b"\x80"
    return (b"\x06" if codec == 264 else b"\x4e\x01") + body


def is_param_set(codec, nal):
    t = nal[0] & 31 if codec == 264 else (nal[0] >> 1) & 63
    return t in ((7, 8) if codec == 264 else (32, 33, 34))


def variants(stream, codec):
    nals = split_nals(stream)
    ps = [x for x in nals if is_param_set(codec, x)]
    rest = [x for x in nals if not is_param_set(codec, x)]
    return {
        "aud_first": join([aud(codec)] + nals),
        "sei_after_ps": join(ps + [sei(codec)] + rest),
        "two_pictures": join(nals + nals),
        "trailing_zeros": join(nals) + b"\x00" * 7,
        "three_byte_start_codes": join(nals, b"\x00\x00\x01"),
    }
