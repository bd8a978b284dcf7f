"""Image output and the comparison statistics of the reference scripts.

Replaces ``mi.util.write_bitmap`` (``path.py:353-354``, ``nrc.py:140``,
``test-restir-spatial.py:24,61,76``, ``restirgi.py:608,626``,
``testpssmlt.py:28``) and ``mi.util.convert_to_bitmap``
(``test-restir-spatial.py:81``): ``.exr`` files are written as OpenEXR
scanline images with 32-bit float R, G, B channels (hdrfilm ``rgb``,
``scene.xml:18-24``), ZIP- or un-compressed; ``.png`` / ``.jpg`` go through
the sRGB transfer curve to 8 bits (Pillow). The statistics mirror
``test-restir-spatial.py:55-57`` (``dr.mean_nested`` of the squared
deviation / difference).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

# ------------------------------------------------------------------ OpenEXR --
_MAGIC = 20000630
_COMPRESSION = {"none": 0, "zips": 2, "zip": 3}
_LINES = {0: 1, 2: 1, 3: 16}


def _attr(name: str, typ: str, data: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _zip_pack(raw: bytes) -> bytes:
    """OpenEXR ZIP: interleave the byte halves, delta-predict, deflate."""
    a = np.frombuffer(raw, np.uint8)
    t = np.empty_like(a)
    half = (len(a) + 1) // 2
    t[:half] = a[0::2]
    t[half:] = a[1::2]
    d = t.astype(np.int16)
    d[1:] = (t[1:].astype(np.int16) - t[:-1].astype(np.int16) + 128) & 0xFF
    return zlib.compress(d.astype(np.uint8).tobytes(), 6)


def _zip_unpack(data: bytes, size: int) -> bytes:
    d = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int32)
    t = np.cumsum(np.concatenate([d[:1], d[1:] - 128])) & 0xFF
    t = t.astype(np.uint8)
    out = np.empty(size, np.uint8)
    half = (size + 1) // 2
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


def write_exr(path: str, img, compression: str = "zip") -> None:
    """Write an [H, W, 3] (or [H, W]) float image as an RGB float32 EXR."""
    img = np.asarray(img, np.float32)
    if img.ndim == 2:
        img = np.repeat(img[..., None], 3, 2)
    H, W, C = img.shape
    if C < 3:
        raise ValueError("need 3 channels")
    comp = _COMPRESSION[compression]
    chans = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", 2, 0, 1, 1) for n in "BGR") + b"\0"
    box = struct.pack("<iiii", 0, 0, W - 1, H - 1)
    header = (struct.pack("<ii", _MAGIC, 2) + _attr("channels", "chlist", chans)
              + _attr("compression", "compression", bytes([comp])) + _attr("dataWindow", "box2i", box)
              + _attr("displayWindow", "box2i", box) + _attr("lineOrder", "lineOrder", b"\0")
              + _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
              + _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
              + _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)) + b"\0")
    lines = _LINES[comp]
    # per scanline: channels in alphabetical order (B, G, R), W floats each
    planar = np.ascontiguousarray(img[..., [2, 1, 0]].transpose(0, 2, 1)).astype("<f4")
    chunks = []
    for y0 in range(0, H, lines):
        raw = planar[y0:y0 + lines].tobytes()
        data = raw
        if comp:
            z = _zip_pack(raw)
            if len(z) < len(raw):
                data = z
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    offset = len(header) + 8 * len(chunks)
    table = []
    for c in chunks:
        table.append(offset)
        offset += len(c)
    with open(path, "wb") as f:
        f.write(header + struct.pack(f"<{len(table)}Q", *table) + b"".join(chunks))


def read_exr(path: str) -> np.ndarray:
    """Read an RGB float32 scanline EXR written by :func:`write_exr` (also
    accepts half-float channels and the NO/ZIPS/ZIP compressions)."""
    buf = open(path, "rb").read()
    magic, _ver = struct.unpack_from("<ii", buf, 0)
    if magic != _MAGIC:
        raise ValueError("not an OpenEXR file")
    pos = 8
    attrs = {}
    while buf[pos] != 0:
        e = buf.index(b"\0", pos)
        name = buf[pos:e].decode()
        e2 = buf.index(b"\0", e + 1)
        (size,) = struct.unpack_from("<i", buf, e2 + 1)
        attrs[name] = buf[e2 + 5:e2 + 5 + size]
        pos = e2 + 5 + size
    pos += 1
    chans, c = [], attrs["channels"]
    i = 0
    while c[i] != 0:
        e = c.index(b"\0", i)
        (pt,) = struct.unpack_from("<i", c, e + 1)
        chans.append((c[i:e].decode(), pt))
        i = e + 17
    comp = attrs["compression"][0]
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    lines = _LINES[comp]
    n_chunks = (H + lines - 1) // lines
    table = struct.unpack_from(f"<{n_chunks}Q", buf, pos)
    bpp = [4 if pt == 2 else 2 for _, pt in chans]
    out = {n: np.zeros((H, W), np.float32) for n, _ in chans}
    for off in table:
        yy, size = struct.unpack_from("<ii", buf, off)
        nl = min(lines, y1 + 1 - yy)
        raw_size = nl * W * sum(bpp)
        data = buf[off + 8:off + 8 + size]
        if comp and size < raw_size:
            data = _zip_unpack(data, raw_size)
        p = 0
        for ln in range(nl):
            for (name, pt), b in zip(chans, bpp):
                v = np.frombuffer(data, "<f4" if b == 4 else "<f2", W, p)
                out[name][yy - y0 + ln] = v
                p += W * b
    return np.stack([out["R"], out["G"], out["B"]], -1)


# ----------------------------------------------------------------- bitmaps --
def convert_to_bitmap(img) -> np.ndarray:
    """Linear RGB -> 8-bit sRGB (mi.util.convert_to_bitmap)."""
    x = np.clip(np.asarray(img, np.float64), 0.0, None)
    s = np.where(x <= 0.0031308, 12.92 * x, 1.055 * np.power(x, 1.0 / 2.4) - 0.055)
    return np.clip(np.round(np.clip(s, 0.0, 1.0) * 255.0), 0, 255).astype(np.uint8)


def write_bitmap(path: str, img) -> None:
    """mi.util.write_bitmap: .exr (float RGB) or an 8-bit sRGB .png/.jpg."""
    img = np.asarray(img)
    if path.lower().endswith(".exr"):
        write_exr(path, img)
        return
    from PIL import Image

    Image.fromarray(convert_to_bitmap(img[..., :3])).save(path)


# -------------------------------------------------------------- statistics --
def mean_nested(x) -> float:
    return float(np.mean(np.asarray(x, np.float64)))


def variance(img) -> float:
    """dr.mean_nested(dr.sqr(img - dr.mean_nested(img))) (test-restir-spatial.py:55)."""
    img = np.asarray(img, np.float64)
    return float(np.mean((img - img.mean()) ** 2))


def bias(img, ref) -> float:
    """dr.mean_nested(img - ref) (test-restir-spatial.py:56)."""
    return float(np.mean(np.asarray(img, np.float64) - np.asarray(ref, np.float64)))


def mse(img, ref) -> float:
    """dr.mean_nested(dr.sqr(img - ref)) (test-restir-spatial.py:57)."""
    return float(np.mean((np.asarray(img, np.float64) - np.asarray(ref, np.float64)) ** 2))
