"""Test-only writers for the SID input path: a PNG encoder (any filter per row, Adam7, 8/16-bit RGB, palettes,
the rejected colour types, split IDAT) and an LMDB 0.9 (64-bit) environment writer (leaf / branch / overflow pages),
so the native reader and decoder can be exercised on more shapes than the reference's two fixtures hold."""
from __future__ import annotations

import struct
import zlib
from typing import Dict, List, Optional

import numpy as np


# --------------------------------------------------------------------------------------------------------- PNG
def _chunk(typ: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + typ + data + struct.pack(">I", zlib.crc32(typ + data))


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def _filter_row(ft: int, row: np.ndarray, prev: np.ndarray, bpp: int) -> bytes:
    r = row.astype(np.int64)
    p = prev.astype(np.int64)
    out = np.zeros_like(r)
    for i in range(len(r)):
        a = r[i - bpp] if i >= bpp else 0
        b = p[i]
        c = p[i - bpp] if i >= bpp else 0
        pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
        out[i] = (r[i] - pred) & 255
    return bytes([ft]) + out.astype(np.uint8).tobytes()


def _pack(samples: np.ndarray, depth: int) -> np.ndarray:
    """[rows][n] integer samples -> [rows][bytes] scanline bytes."""
    if depth == 16:
        s = samples.astype(np.uint16)
        return np.stack([(s >> 8).astype(np.uint8), (s & 255).astype(np.uint8)], -1).reshape(s.shape[0], -1)
    if depth == 8:
        return samples.astype(np.uint8)
    bits = ((samples[..., None] >> np.arange(depth - 1, -1, -1)) & 1).astype(np.uint8)
    bits = bits.reshape(samples.shape[0], -1)
    pad = (-bits.shape[1]) % 8
    bits = np.pad(bits, ((0, 0), (0, pad)))
    return np.packbits(bits, axis=1)


def encode_png(samples: np.ndarray, depth: int, ctype: int, palette: Optional[np.ndarray] = None,
               interlace: bool = False, filters=None, trns: bool = False, idat_split: int = 0,
               rng: Optional[np.random.Generator] = None) -> bytes:
    """samples: [H][W][spp] integers (palette indices for ctype 3).  filters: None = random per row, or an int."""
    H, W = samples.shape[:2]
    spp = samples.shape[2]
    bpp = max(1, spp * depth // 8)
    rng = rng or np.random.default_rng(0)
    passes = [(0, 0, 1, 1)] if not interlace else \
        [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
    raw = b""
    for xs, ys, dx, dy in passes:
        sub = samples[ys::dy, xs::dx]
        if sub.size == 0:
            continue
        rows = _pack(sub.reshape(sub.shape[0], -1), depth)
        prev = np.zeros(rows.shape[1], np.uint8)
        for y in range(rows.shape[0]):
            ft = int(rng.integers(0, 5)) if filters is None else int(filters)
            raw += _filter_row(ft, rows[y], prev, bpp)
            prev = rows[y]
    z = zlib.compress(raw, 6)
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        out += _chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    if trns:
        out += _chunk(b"tRNS", b"\x00")
    out += _chunk(b"tEXt", b"Comment\x00ancillary chunk")
    if idat_split:
        for i in range(0, len(z), idat_split):
            out += _chunk(b"IDAT", z[i:i + idat_split])
    else:
        out += _chunk(b"IDAT", z)
    return out + _chunk(b"IEND", b"")


# -------------------------------------------------------------------------------------------------------- LMDB
PS = 4096


def _page_header(pgno: int, flags: int, lower: int = 0, upper: int = 0) -> bytearray:
    page = bytearray(PS)
    struct.pack_into("<QHHHH", page, 0, pgno, 0, flags, lower, upper)
    return page


def _put_nodes(page: bytearray, nodes: List[bytes]) -> None:
    upper = PS
    for i, nd in enumerate(nodes):
        upper -= len(nd) + (len(nd) & 1)
        page[upper:upper + len(nd)] = nd
        struct.pack_into("<H", page, 16 + 2 * i, upper)
    struct.pack_into("<HH", page, 12, 16 + 2 * len(nodes), upper)


def write_lmdb(path: str, items: Dict[bytes, bytes], inline_max: int = 600, leaf_fill: int = 3000,
               fanout: Optional[int] = None) -> None:
    """Write `items` as an LMDB environment file (data.mdb layout): sorted leaves (values above `inline_max` bytes on
    overflow pages), then branch levels until one root remains.  `fanout` caps the children per branch page."""
    pages: List[bytearray] = [bytearray(PS), bytearray(PS)]  # meta pages, filled last
    keys = sorted(items)
    leaves: List[List[bytes]] = [[]]
    leaf_first: List[bytes] = []
    size = 0
    overflow = 0
    for k in keys:
        v = items[k]
        if len(v) > inline_max:
            n = (16 + len(v) + PS - 1) // PS
            pg = len(pages)
            first = _page_header(pg, 0x04)
            struct.pack_into("<I", first, 12, n)
            blob = bytes(first[:16]) + v
            blob += b"\x00" * (n * PS - len(blob))
            for j in range(n):
                pages.append(bytearray(blob[j * PS:(j + 1) * PS]))
            overflow += n
            nd = struct.pack("<HHHH", len(v) & 0xFFFF, len(v) >> 16, 0x01, len(k)) + k + struct.pack("<Q", pg)
        else:
            nd = struct.pack("<HHHH", len(v) & 0xFFFF, len(v) >> 16, 0, len(k)) + k + v
        cost = len(nd) + (len(nd) & 1) + 2
        if leaves[-1] and size + cost > leaf_fill:
            leaves.append([])
            size = 0
        if not leaves[-1]:
            leaf_first.append(k)
        leaves[-1].append(nd)
        size += cost
    level = []
    for nodes, k0 in zip(leaves, leaf_first):
        pg = len(pages)
        page = _page_header(pg, 0x02)
        _put_nodes(page, nodes)
        pages.append(page)
        level.append((k0, pg))
    depth, branch_pages = 1, 0
    cap = fanout or 100
    while len(level) > 1:
        nxt = []
        for i in range(0, len(level), cap):
            group = level[i:i + cap]
            nodes = []
            for j, (k, child) in enumerate(group):
                key = b"" if j == 0 else k
                nodes.append(struct.pack("<HHHH", child & 0xFFFF, (child >> 16) & 0xFFFF, (child >> 32) & 0xFFFF,
                                         len(key)) + key)
            pg = len(pages)
            page = _page_header(pg, 0x01)
            _put_nodes(page, nodes)
            pages.append(page)
            nxt.append((group[0][0], pg))
            branch_pages += 1
        level = nxt
        depth += 1
    root = level[0][1] if items else 2 ** 64 - 1
    for i in range(2):
        meta = _page_header(i, 0x08)
        free_db = struct.pack("<IHHQQQQQ", PS, 0, 0, 0, 0, 0, 0, 2 ** 64 - 1)
        main_db = struct.pack("<IHHQQQQQ", 0, 0, depth if items else 0, branch_pages, len(leaves) if items else 0,
                              overflow, len(items), root)
        body = struct.pack("<IIQQ", 0xBEEFC0DE, 1, 0, 1 << 30) + free_db + main_db + \
            struct.pack("<QQ", len(pages) - 1, i + 1)  # meta 1 is the newer one
        meta[16:16 + len(body)] = body
        pages[i] = meta
    with open(path, "wb") as f:
        for p in pages:
            f.write(bytes(p))
