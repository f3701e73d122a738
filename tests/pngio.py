"""Minimal PNG reader/writer (8-bit RGB/RGBA/gray) used by tests to load gallery images and
rendered outputs without third-party imaging libraries."""
import struct
import zlib

import numpy as np


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def read_png(path):
    """Return uint8 array [H, W, C] in file (top-down) row order."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n", path
    pos = 8
    idat = b""
    w = h = bitdepth = ctype = None
    while pos < len(data):
        (ln,) = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + ln]
        pos += 12 + ln
        if typ == b"IHDR":
            w, h, bitdepth, ctype = struct.unpack(">IIBB", body[:10])
            assert body[12] == 0, "interlaced PNG not supported"
        elif typ == b"IDAT":
            idat += body
        elif typ == b"IEND":
            break
    assert bitdepth == 8, bitdepth
    nch = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    raw = zlib.decompress(idat)
    stride = w * nch
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    off = 0
    for y in range(h):
        ft = raw[off]
        line = np.frombuffer(raw[off + 1:off + 1 + stride], dtype=np.uint8).astype(np.int32)
        off += 1 + stride
        cur = line.copy()
        if ft == 1:
            for i in range(nch, stride):
                cur[i] = (cur[i] + cur[i - nch]) & 255
        elif ft == 2:
            cur = (line + prev) & 255
        elif ft == 3:
            for i in range(stride):
                left = cur[i - nch] if i >= nch else 0
                cur[i] = (line[i] + ((left + prev[i]) >> 1)) & 255
        elif ft == 4:
            for i in range(stride):
                left = cur[i - nch] if i >= nch else 0
                upleft = prev[i - nch] if i >= nch else 0
                cur[i] = (line[i] + _paeth(left, prev[i], upleft)) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, nch)


def write_png(path, img):
    """img: uint8 [H, W, 3] top-down."""
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, b):
        c = struct.pack(">I", len(b)) + t + b
        return c + struct.pack(">I", zlib.crc32(t + b) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))
