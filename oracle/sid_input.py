"""Oracle (test infrastructure only) for the SID input path.

Only tests/ (and bench / smoke checkers) may import this module; the product path is
lowlight_image_enhancement_amd/data (C++ decode + HIP conversion) and never calls it.

CPU restatement of the reference's per-sample input arithmetic and of the two third-party formats it reads through
absent libraries:
  * ``getitem_arrays`` — NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py:196-251 (``__getitem__``):
    uint16 -> float32 / 65535, ``clip(short_raw * expo_ratio, 0, 1)``, ``_maybe_random_crop`` (:162-192) with the
    dataset's ``numpy.random.default_rng(seed)`` draws, then ``img2tensor`` HWC -> CHW float32.
  * ``png_decode`` — what ``_load_png_uint16`` (:38-56) gets from ``cv2.imdecode(buf, IMREAD_UNCHANGED)`` followed
    by the uint8 -> uint16 ``* 257`` promotion and BGR2RGB (net: the file's R, G, B order).  cv2 / libpng are not in
    this image; this is the PNG specification (ISO/IEC 15948: zlib stream, filters 0-4, Adam7, palette expansion)
    restated with zlib + numpy.  Pinned against PIL on the reference's fixture PNGs (data/debug_sid) and on
    synthetic images PIL can decode.
  * ``LmdbReader`` — ``lmdb==`` (py-lmdb, not installed here) ``txn.get(key)`` as used by basicsr's FileClient
    'lmdb' backend, restated from LMDB 0.9's on-disk format (64-bit): meta pages 0/1 (newest txnid wins), main-db
    root, branch / leaf node search with the default memcmp-then-length key order, overflow pages for large values.
    Pinned against the reference's fixture environments (data/debug_sid/*.lmdb), whose PNG values decode to the
    same pixels as the matching files on disk.
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Dict, Optional, Tuple

import numpy as np

MAX_16BIT_VALUE = 65535.0


# ----------------------------------------------------------------------------------------------------------- PNG
def _paeth(a: int, b: int, c: int) -> int:
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _unfilter(raw: bytes, rows: int, rb: int, bpp: int) -> np.ndarray:
    """Reconstruct `rows` filtered scanlines of `rb` bytes (each preceded by its filter byte)."""
    out = np.zeros((rows, rb), np.uint8)
    prev = np.zeros(rb, np.int64)
    for y in range(rows):
        ft = raw[y * (rb + 1)]
        cur = np.frombuffer(raw, np.uint8, rb, y * (rb + 1) + 1).astype(np.int64)
        if ft == 0:
            rec = cur
        elif ft == 2:
            rec = (cur + prev) & 255
        elif ft in (1, 3, 4):
            rec = np.zeros(rb, np.int64)
            for i in range(rb):
                a = int(rec[i - bpp]) if i >= bpp else 0
                b = int(prev[i])
                c = int(prev[i - bpp]) if i >= bpp else 0
                pred = a if ft == 1 else ((a + b) >> 1 if ft == 3 else _paeth(a, b, c))
                rec[i] = (int(cur[i]) + pred) & 255
        else:
            raise ValueError(f"PNG: bad filter type {ft}")
        out[y] = rec
        prev = rec
    return out


def _samples(rows: np.ndarray, depth: int, count: int) -> np.ndarray:
    """Scanline bytes -> `count` integer samples per row (big-endian 16-bit, packed sub-byte depths)."""
    if depth == 16:
        return (rows[:, 0:2 * count:2].astype(np.uint32) << 8) | rows[:, 1:2 * count:2]
    if depth == 8:
        return rows[:, :count].astype(np.uint32)
    bits = np.unpackbits(rows, axis=1)[:, :count * depth].reshape(rows.shape[0], count, depth)
    weights = (1 << np.arange(depth - 1, -1, -1)).astype(np.uint32)
    return (bits.astype(np.uint32) * weights).sum(-1).astype(np.uint32)


def png_parse(buf: bytes) -> Dict:
    if buf is None or len(buf) < 8 or buf[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("PNG: bad signature")
    pos, info, idat = 8, {}, []
    while pos + 12 <= len(buf):
        n, typ = struct.unpack(">I4s", buf[pos:pos + 8])
        data = buf[pos + 8:pos + 8 + n]
        if len(data) != n or pos + 12 + n > len(buf):
            raise ValueError("PNG: truncated chunk")
        (crc,) = struct.unpack(">I", buf[pos + 8 + n:pos + 12 + n])
        if zlib.crc32(typ + data) != crc:
            if not typ[0] & 0x20:  # critical chunk: error; ancillary: discarded (libpng's default)
                raise ValueError("PNG: CRC mismatch")
            pos += 12 + n
            continue
        if typ == b"IHDR":
            w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", data)
            info.update(w=w, h=h, depth=depth, ctype=ctype, interlace=inter)
        elif typ == b"PLTE":
            info["plte"] = np.frombuffer(data, np.uint8).reshape(-1, 3)
        elif typ == b"tRNS":
            info["trns"] = True
        elif typ == b"IDAT":
            idat.append(data)
        elif typ == b"IEND":
            break
        pos += 12 + n
    info["data"] = b"".join(idat)
    return info


def cv2_channels(info: Dict) -> int:
    """Channels of cv2.imdecode(IMREAD_UNCHANGED): gray 1, RGB 3, palette 3 (4 with tRNS), alpha forms 4."""
    return {0: 1, 2: 3, 3: 4 if info.get("trns") else 3}.get(info["ctype"], 4)


def png_decode(buf: bytes) -> np.ndarray:
    """3-channel PNG -> uint16 [H][W][3], file channel order, 8-bit values * 257 (raises ValueError otherwise)."""
    info = png_parse(buf)
    if cv2_channels(info) != 3:
        raise ValueError(f"PNG: {cv2_channels(info)}-channel image (3 expected)")
    H, W, depth, ctype = info["h"], info["w"], info["depth"], info["ctype"]
    spp = 3 if ctype == 2 else 1
    bpp = max(1, spp * depth // 8)
    raw = zlib.decompress(info["data"])
    img = np.zeros((H, W, spp), np.uint32)
    passes = [(0, 0, 1, 1)] if not info["interlace"] else \
        [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
    off = 0
    for xs, ys, dx, dy in passes:
        pw, ph = (W - xs + dx - 1) // dx, (H - ys + dy - 1) // dy
        if pw <= 0 or ph <= 0:
            continue
        rb = (pw * spp * depth + 7) // 8
        need = ph * (rb + 1)
        if off + need > len(raw):
            raise ValueError("PNG: truncated image data")
        rows = _unfilter(raw[off:off + need], ph, rb, bpp)
        off += need
        img[ys::dy, xs::dx] = _samples(rows, depth, pw * spp).reshape(ph, pw, spp)
    if ctype == 3:
        plte = info["plte"].astype(np.uint32)
        if img.max() >= len(plte):
            raise ValueError("PNG: palette index out of range")
        return (plte[img[..., 0]] * 257).astype(np.uint16)
    return (img if depth == 16 else img * 257).astype(np.uint16)


# ---------------------------------------------------------------------------------------------------------- LMDB
class LmdbReader:
    """Read-only key lookup in an LMDB 0.9 environment (64-bit layout); get() returns bytes or None."""

    P_BRANCH, P_LEAF, P_OVERFLOW, P_META = 0x01, 0x02, 0x04, 0x08
    F_BIGDATA = 0x01

    def __init__(self, path: str):
        if os.path.isdir(path):
            path = os.path.join(path, "data.mdb")
        with open(path, "rb") as f:
            self.buf = f.read()
        self.psize = struct.unpack_from("<I", self.buf, 16 + 24)[0]
        best = None
        for i in range(2):
            p = i * self.psize
            flags = struct.unpack_from("<H", self.buf, p + 10)[0]
            magic, version = struct.unpack_from("<II", self.buf, p + 16)
            if not flags & self.P_META or magic != 0xBEEFC0DE or version != 1:
                continue
            txn = struct.unpack_from("<Q", self.buf, p + 16 + 24 + 96 + 8)[0]
            if best is None or txn > best[0]:
                best = (txn, p)
        if best is None:
            raise ValueError("not an LMDB data file")
        main = best[1] + 16 + 24 + 48
        self.entries = struct.unpack_from("<Q", self.buf, main + 32)[0]
        self.root = struct.unpack_from("<Q", self.buf, main + 40)[0]

    def _nodes(self, pg: int):
        p = pg * self.psize
        flags, lower = struct.unpack_from("<HH", self.buf, p + 10)
        out = []
        for i in range((lower - 16) // 2):
            off = struct.unpack_from("<H", self.buf, p + 16 + 2 * i)[0]
            lo, hi, nflags, ks = struct.unpack_from("<HHHH", self.buf, p + off)
            key = self.buf[p + off + 8:p + off + 8 + ks]
            out.append((lo, hi, nflags, key, p + off + 8 + ks))
        return flags, out

    def get(self, key: bytes) -> Optional[bytes]:
        pg = self.root
        if pg == 2 ** 64 - 1:
            return None
        while True:
            flags, nodes = self._nodes(pg)
            if flags & self.P_BRANCH:
                pick = 0
                for i in range(1, len(nodes)):  # last child whose separator key <= key (memcmp, then length)
                    if nodes[i][3] <= key:
                        pick = i
                lo, hi, nf, _, _ = nodes[pick]
                pg = lo | (hi << 16) | (nf << 32)
                continue
            for lo, hi, nf, k, data in nodes:
                if k == key:
                    size = lo | (hi << 16)
                    if nf & self.F_BIGDATA:
                        opg = struct.unpack_from("<Q", self.buf, data)[0]
                        start = opg * self.psize + 16
                        return self.buf[start:start + size]
                    return self.buf[data:data + size]
            return None


# ----------------------------------------------------------------------------------------------- __getitem__ math
def crop_window(rng: np.random.Generator, h: int, w: int, ps: Optional[int], phase: str, random_crop: bool
                ) -> Tuple[int, int, int, int]:
    """_maybe_random_crop's (top, left, height, width) (sony_sid_lmdb_dataset.py:162-192), drawing from `rng`."""
    if ps is None or phase != "train":
        return 0, 0, h, w
    if ps > h or ps > w:
        raise ValueError(f"Patch size {ps} exceeds source dimensions {(h, w)}.")
    if random_crop:
        top = int(rng.integers(0, h - ps + 1))
        left = int(rng.integers(0, w - ps + 1))
    else:
        top, left = (h - ps) // 2, (w - ps) // 2
    return top, left, ps, ps


def getitem_arrays(short_u16: np.ndarray, long_u16: np.ndarray, expo_ratio: float, window) -> Dict[str, np.ndarray]:
    """sony_sid_lmdb_dataset.py:207-229 on HWC uint16 arrays: float32 CHW lq / gt / short_raw / long_raw."""
    short_raw = short_u16.astype(np.float32) / MAX_16BIT_VALUE
    long_raw = long_u16.astype(np.float32) / MAX_16BIT_VALUE
    aligned = np.clip(short_raw * expo_ratio, 0.0, 1.0)
    top, left, ch, cw = window
    crop = lambda a: a[top:top + ch, left:left + cw, :]  # noqa: E731
    chw = lambda a: np.ascontiguousarray(crop(a).transpose(2, 0, 1)).astype(np.float32)  # noqa: E731
    return {"lq": chw(aligned), "gt": chw(long_raw), "short_raw": chw(short_raw), "long_raw": chw(long_raw)}
