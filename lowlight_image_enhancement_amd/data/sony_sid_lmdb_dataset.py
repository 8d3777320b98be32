"""Sony SID dataset (LMDB or disk), MI355X input path.

Reference: NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py.  Same options, manifest filtering, exceptions, crop
draws (``numpy.random.default_rng(seed)``: ``top`` then ``left`` per training sample) and batch contract.  The work
is split differently:

  * host, native (liblowlight_nbp.so, sid_io.cpp): LMDB lookup (mmap, no lmdb package), PNG decode (zlib) straight
    into the crop window as uint16 — ``__getitem__`` returns the cropped uint16 HWC arrays (``lq_u16`` / ``gt_u16``),
    the ratio and the string fields; ``get_batch`` decodes a whole batch on host threads;
  * device (sid.hip, ``nbp_sid_to_float``): ``/ 65535``, ``clip(short * ratio, 0, 1)`` and HWC -> CHW, run by
    ``CUDAPrefetcher`` (prefetch_dataloader.py) on its side stream, which hands the training step the reference's
    batch dict (``lq``, ``gt``, ``short``, ``long``, ``short_raw``, ``long_raw``, ``short_obs``, ``expo_ratio``, ...).

Only the crop window crosses PCIe, as uint16: 1/4 of the float32 bytes of the reference's per-sample tensors
(which also carry ``short_raw`` and ``long_raw``).  The arithmetic is bit-identical to the reference's numpy float32
(tests/test_sid_input.py).
"""
from __future__ import annotations

import ctypes
import json
import os
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch.utils import data as torch_data

from .._lib import NBPError, host_call
from .file_client import FileClient, expand_with_sid_root

MAX_16BIT_VALUE = 65535.0


def _expand_to_path(path_value: Union[str, os.PathLike]) -> Path:
    path = expand_with_sid_root(path_value)
    if path is None:
        raise ValueError("Received an empty path while resolving dataset inputs.")
    return path


def png_shape(buffer: bytes) -> Tuple[int, int, int]:
    """(H, W, C) of the array cv2.imdecode(IMREAD_UNCHANGED) would return for this PNG (IHDR only)."""
    if buffer is None:
        raise ValueError("Received empty buffer when decoding PNG.")
    h, w, c, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    try:
        host_call("png_info", buffer, len(buffer), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c), ctypes.byref(d))
    except NBPError as e:
        raise ValueError("Failed to decode PNG buffer into an image.") from e
    return h.value, w.value, c.value


def _check_three_channels(shape: Tuple[int, int, int]) -> None:
    if shape[2] != 3:
        raise ValueError(f"Expected 3-channel image, got shape {shape}.")


def _load_png_uint16(buffer: bytes, window: Optional[Tuple[int, int, int, int]] = None) -> np.ndarray:
    """sony_sid_lmdb_dataset.py:38-56: PNG bytes -> uint16 HWC in RGB order (uint8 promoted by * 257).
    `window` = (top, left, height, width) decodes only that crop."""
    shape = png_shape(buffer)
    _check_three_channels(shape)
    top, left, ch, cw = window if window is not None else (0, 0, shape[0], shape[1])
    out = np.empty((ch, cw, 3), np.uint16)
    try:
        host_call("png_decode_rgb16", buffer, len(buffer), out.ctypes.data, top, left, ch, cw)
    except NBPError as e:
        raise ValueError("Failed to decode PNG buffer into an image.") from e
    return out


def decode_batch(buffers: Sequence[bytes], windows: Sequence[Tuple[int, int, int, int]], nthreads: int = 8
                 ) -> np.ndarray:
    """Decode n PNGs into their (common-size) crop windows on `nthreads` native threads: uint16 [n][h][w][3]."""
    n = len(buffers)
    if n == 0:
        raise ValueError("decode_batch: empty batch")
    ch, cw = windows[0][2], windows[0][3]
    if any(w[2] != ch or w[3] != cw for w in windows):
        raise ValueError("decode_batch: the crop windows of a batch must have one size")
    for b in buffers:
        _check_three_channels(png_shape(b))
    out = np.empty((n, ch, cw, 3), np.uint16)
    keep = [ctypes.c_char_p(b) for b in buffers]
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(k, ctypes.c_void_p).value for k in keep])
    lens = (ctypes.c_long * n)(*[len(b) for b in buffers])
    tops = (ctypes.c_int * n)(*[w[0] for w in windows])
    lefts = (ctypes.c_int * n)(*[w[1] for w in windows])
    try:
        host_call("png_decode_batch", n, ptrs, lens, tops, lefts, ch, cw, out.ctypes.data, int(nthreads))
    except NBPError as e:
        raise ValueError(f"Failed to decode PNG buffer into an image: {e}") from e
    return out


def _u16_tensor(a: np.ndarray) -> torch.Tensor:
    """uint16 array -> int16-typed CPU tensor of the same bits (collatable, pinnable); the device kernel reads it
    as uint16."""
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16))


class SonySIDLMDBDataset(torch_data.Dataset):
    """Sony SID dataset backed by LMDB (or disk); see the module docstring for the sample format."""

    def __init__(self, opt: dict):
        super().__init__()
        self.opt = opt
        self.phase: str = opt.get("phase", "train")
        self.patch_size: Optional[int] = opt.get("patch_size")
        self.samples_per_pair: int = int(opt.get("samples_per_pair", 1))
        self.random_crop: bool = opt.get("random_crop", True)
        self.return_metadata: bool = opt.get("return_metadata", False)
        self.rng = np.random.default_rng(opt.get("seed", None))

        manifest_path = _expand_to_path(opt["manifest_path"])
        if not manifest_path.is_file():
            raise FileNotFoundError(f"Manifest file not found: {manifest_path}")
        with manifest_path.open("r", encoding="utf-8") as f:
            manifest_data = json.load(f)

        subset = opt.get("subset", self.phase)
        self.subset = subset
        allowed_ids = set(opt.get("allowed_pair_ids", []))
        entries: List[dict] = []
        for record in manifest_data:
            if record.get("subset") != subset:
                continue
            if allowed_ids and record["pair_id"] not in allowed_ids:
                continue
            entries.append(record)
        if not entries:
            raise RuntimeError(f"No entries available for subset='{subset}'.")
        self.entries = entries
        self._num_pairs = len(entries)

        io_backend_opt = dict(opt.get("io_backend", {}))
        if not io_backend_opt and ("short_lmdb" in opt or "long_lmdb" in opt):
            io_backend_opt = {"type": "lmdb", "db_paths": [opt.get("short_lmdb"), opt.get("long_lmdb")],
                              "client_keys": ["short", "long"]}
        if not io_backend_opt:
            raise KeyError("Dataset option must provide 'io_backend' or 'short_lmdb'/'long_lmdb' paths.")
        self.file_client: Optional[FileClient] = None
        backend_type = io_backend_opt.pop("type")
        self.io_backend_type = backend_type
        if backend_type == "lmdb":
            db_paths = io_backend_opt.get("db_paths")
            client_keys = io_backend_opt.get("client_keys")
            if not db_paths or not client_keys:
                raise KeyError("LMDB backend requires 'db_paths' and 'client_keys'.")
            if any(not p for p in db_paths):
                raise ValueError(f"Invalid LMDB paths provided: {db_paths}")
            db_paths = [_expand_to_path(p) for p in db_paths]
            self.file_client = FileClient(backend="lmdb", db_paths=[str(p) for p in db_paths],
                                          client_keys=client_keys, readonly=True, lock=False, readahead=False)
        elif backend_type == "disk":
            self.root_short = _expand_to_path(io_backend_opt["paths"]["short"])
            self.root_long = _expand_to_path(io_backend_opt["paths"]["long"])
            if not self.root_short.is_dir() or not self.root_long.is_dir():
                raise FileNotFoundError(
                    f"Disk backend paths must exist. short={self.root_short}, long={self.root_long}")
        else:
            raise ValueError(f"Unsupported io_backend type: {backend_type}")

    def __len__(self) -> int:
        return self._num_pairs * self.samples_per_pair

    def _fetch_bytes(self, key: str, *, client_key: str) -> Optional[bytes]:
        if self.io_backend_type == "lmdb":
            assert self.file_client is not None
            return self.file_client.get(key, client_key=client_key)
        root = self.root_short if client_key == "short" else self.root_long
        with (root / key).open("rb") as f:
            return f.read()

    def _crop_window(self, h: int, w: int) -> Tuple[int, int, int, int]:
        """_maybe_random_crop (:162-192): the window, drawing top then left from self.rng."""
        if self.patch_size is None or self.phase != "train":
            return 0, 0, h, w
        ps = self.patch_size
        if ps > h or ps > w:
            raise ValueError(f"Patch size {ps} exceeds source dimensions {(h, w)}.")
        if self.random_crop:
            top = self.rng.integers(0, h - ps + 1)
            left = self.rng.integers(0, w - ps + 1)
        else:
            top, left = (h - ps) // 2, (w - ps) // 2
        return int(top), int(left), ps, ps

    def _prepare(self, index: int):
        entry = self.entries[index // self.samples_per_pair]
        short_buf = self._fetch_bytes(entry["short_key"], client_key="short")
        long_buf = self._fetch_bytes(entry["long_key"], client_key="long")
        short_shape, long_shape = png_shape(short_buf), png_shape(long_buf)
        _check_three_channels(short_shape)
        _check_three_channels(long_shape)
        window = self._crop_window(short_shape[0], short_shape[1])
        if window[0] + window[2] > long_shape[0] or window[1] + window[3] > long_shape[1]:
            raise ValueError(f"Long-exposure image {long_shape} is smaller than the crop window {window}.")
        return entry, short_buf, long_buf, window

    def _fields(self, entry: dict) -> Dict:
        expo_ratio = float(entry["exposure_ratio"])
        pair_id = entry["pair_id"]
        sample = {"expo_ratio": torch.full((1, 1, 1), expo_ratio, dtype=torch.float32), "pair_id": pair_id,
                  "lq_path": entry["short_key"], "gt_path": entry["long_key"], "key": str(pair_id)}
        if self.return_metadata:
            sample["metadata"] = {"pair_id": pair_id, "short_key": entry["short_key"], "long_key": entry["long_key"],
                                  "subset": entry.get("subset"), "short_exposure": entry.get("short_exposure"),
                                  "long_exposure": entry.get("long_exposure"), "exposure_ratio": expo_ratio}
        return sample

    def __getitem__(self, index: int) -> dict:
        entry, short_buf, long_buf, window = self._prepare(index)
        sample = self._fields(entry)
        sample["lq_u16"] = _u16_tensor(_load_png_uint16(short_buf, window))
        sample["gt_u16"] = _u16_tensor(_load_png_uint16(long_buf, window))
        return sample

    def get_batch(self, indices: Sequence[int], nthreads: int = 8) -> dict:
        """A collated batch (the DataLoader's default_collate of __getitem__ over `indices`, same crop draws in the
        same order) with all 2n PNGs decoded on `nthreads` native threads in one call."""
        prepared = [self._prepare(i) for i in indices]
        bufs = [p[1] for p in prepared] + [p[2] for p in prepared]
        wins = [p[3] for p in prepared] * 2
        u16 = decode_batch(bufs, wins, nthreads)
        n = len(prepared)
        batch = torch_data.default_collate([self._fields(p[0]) for p in prepared])
        batch["lq_u16"] = _u16_tensor(u16[:n])
        batch["gt_u16"] = _u16_tensor(u16[n:])
        return batch
