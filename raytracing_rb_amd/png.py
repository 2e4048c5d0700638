"""Minimal PNG codec (zlib only) for textures in and frames out.

Decoding follows what the reference's texture loader sees through RMagick
(``src/objects/texture.rb:12-20``): every sample as a 16-bit quantum, of which
``>> 8`` is kept — i.e. the high byte of 16-bit samples and the sample itself
for 8-bit images.  Encoding writes the 8-bit RGBA image the png gem produces in
``Camera#save_image`` (``src/camera.rb:36-39``).
"""

import struct
import zlib

import numpy as np

_SIG = b"\x89PNG\r\n\x1a\n"


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _unfilter(raw, width, height, bpp, stride):
    out = bytearray(height * stride)
    prev = bytearray(stride)
    pos = 0
    for y in range(height):
        ft = raw[pos]
        line = bytearray(raw[pos + 1:pos + 1 + stride])
        pos += 1 + stride
        if ft == 1:
            for i in range(bpp, stride):
                line[i] = (line[i] + line[i - bpp]) & 0xFF
        elif ft == 2:
            for i in range(stride):
                line[i] = (line[i] + prev[i]) & 0xFF
        elif ft == 3:
            for i in range(stride):
                a = line[i - bpp] if i >= bpp else 0
                line[i] = (line[i] + ((a + prev[i]) >> 1)) & 0xFF
        elif ft == 4:
            for i in range(stride):
                a = line[i - bpp] if i >= bpp else 0
                c = prev[i - bpp] if i >= bpp else 0
                line[i] = (line[i] + _paeth(a, prev[i], c)) & 0xFF
        elif ft != 0:
            raise ValueError("bad PNG filter type %d" % ft)
        out[y * stride:(y + 1) * stride] = line
        prev = line
    return bytes(out)


def decode_rgb8(path_or_bytes):
    """Decode a PNG to an (H, W, 3) uint8 array, rows top-down (texture.rb:16-20)."""
    data = path_or_bytes
    if isinstance(path_or_bytes, str):
        with open(path_or_bytes, "rb") as f:
            data = f.read()
    if data[:8] != _SIG:
        raise ValueError("not a PNG file")
    pos = 8
    idat = []
    palette = None
    w = h = depth = ctype = interlace = None
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if tag == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
        elif tag == b"PLTE":
            palette = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif tag == b"IDAT":
            idat.append(body)
        elif tag == b"IEND":
            break
    if interlace:
        raise ValueError("interlaced PNG not supported")
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bits = depth * chans
    bpp = max(1, bits // 8)
    stride = (w * bits + 7) // 8
    raw = _unfilter(zlib.decompress(b"".join(idat)), w, h, bpp, stride)
    if depth == 16:
        a = np.frombuffer(raw, ">u2").reshape(h, w, chans)
        a = (a >> 8).astype(np.uint8)                     # RMagick quantum >> 8
    elif depth == 8:
        a = np.frombuffer(raw, np.uint8).reshape(h, w, chans)
    else:                                                 # 1/2/4-bit gray or palette
        rows = np.frombuffer(raw, np.uint8).reshape(h, stride)
        bitsarr = np.unpackbits(rows, axis=1).reshape(h, stride * 8 // depth, depth)
        vals = np.zeros(bitsarr.shape[:2], np.uint16)
        for k in range(depth):
            vals = (vals << 1) | bitsarr[:, :, k]
        vals = vals[:, :w]
        if ctype == 0:
            vals = vals * (255 // ((1 << depth) - 1))
        a = vals.astype(np.uint8)[:, :, None]
    if ctype == 3:
        return palette[a[:, :, 0]].copy()
    if chans in (1, 2):
        return np.repeat(a[:, :, :1], 3, axis=2).copy()
    return a[:, :, :3].copy()


def _chunk(tag, body):
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF)


def encode(img):
    """Encode an (H, W, 3|4) uint8 array (rows top-down) as an 8-bit PNG; 16-bit if uint16."""
    img = np.ascontiguousarray(img)
    h, w, c = img.shape
    ctype = {3: 2, 4: 6}[c]
    depth = 16 if img.dtype == np.uint16 else 8
    rows = img.astype(">u2").tobytes() if depth == 16 else img.astype(np.uint8).tobytes()
    stride = w * c * depth // 8
    raw = b"".join(b"\x00" + rows[y * stride:(y + 1) * stride] for y in range(h))
    return (_SIG + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
            + _chunk(b"IDAT", zlib.compress(raw, 6)) + _chunk(b"IEND", b""))


def write(path, img):
    with open(path, "wb") as f:
        f.write(encode(img))
