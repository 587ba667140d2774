"""A small PNG decoder for the tests (8-bit greyscale / RGB / RGBA,
non-interlaced), independent of the library's writer: chunk walk with CRC
checks, zlib inflate, per-row unfiltering (None/Sub/Up/Average/Paeth)."""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIGNATURE = b"\x89PNG\r\n\x1a\n"
CHANNELS = {0: 1, 2: 3, 6: 4}


def chunks(data: bytes):
    """Yield (type, payload) with every CRC checked."""
    if data[:8] != SIGNATURE:
        raise ValueError("not a PNG signature")
    pos = 8
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        if zlib.crc32(typ + body) & 0xFFFFFFFF != crc:
            raise ValueError(f"bad CRC in {typ!r}")
        yield typ.decode("ascii"), body
        pos += 12 + n


def decode(data: bytes) -> tuple[np.ndarray, dict]:
    """-> (uint8 (H, W, C), info: ihdr fields + the filter type of each row)."""
    ihdr, idat, ended = None, [], False
    for typ, body in chunks(data):
        if typ == "IHDR":
            w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", body)
            ihdr = dict(width=w, height=h, depth=depth, color_type=ctype, compression=comp, filter=filt,
                        interlace=inter)
        elif typ == "IDAT":
            idat.append(body)
        elif typ == "IEND":
            ended = True
    if ihdr is None or not ended:
        raise ValueError("missing IHDR or IEND")
    if ihdr["depth"] != 8 or ihdr["interlace"] != 0 or ihdr["color_type"] not in CHANNELS:
        raise ValueError(f"unsupported PNG {ihdr}")
    w, h, c = ihdr["width"], ihdr["height"], CHANNELS[ihdr["color_type"]]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8)
    stride = w * c
    if raw.size != h * (stride + 1):
        raise ValueError("IDAT size does not match the image")
    rows = raw.reshape(h, stride + 1)
    out = np.zeros((h, stride), np.int64)
    prev = np.zeros(stride, np.int64)
    filters = rows[:, 0].tolist()
    for y in range(h):
        f, line = filters[y], rows[y, 1:].astype(np.int64)
        cur = np.zeros(stride, np.int64)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            for i in range(stride):
                a = cur[i - c] if i >= c else 0
                b = prev[i]
                cc = prev[i - c] if i >= c else 0
                if f == 1:
                    pred = a
                elif f == 3:
                    pred = (a + b) >> 1
                elif f == 4:
                    p = a + b - cc
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - cc)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else cc)
                else:
                    raise ValueError(f"bad filter type {f}")
                cur[i] = (line[i] + pred) & 255
        out[y] = cur
        prev = cur
    ihdr["row_filters"] = filters
    return out.astype(np.uint8).reshape(h, w, c), ihdr
