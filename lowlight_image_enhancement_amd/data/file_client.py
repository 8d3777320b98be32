"""Storage backends for the SID input path: basicsr's FileClient interface ('lmdb' and 'disk').

Reference: NAFNet_base/basicsr/utils/file_client.py (LmdbBackend :120-185, HardDiskBackend, FileClient :188-225).
The LMDB backend reads the environment through the native read-only reader of liblowlight_nbp.so
(``nbp_lmdb_open`` / ``nbp_lmdb_get``: mmap + B+tree lookup, no lmdb package), so ``get`` returns the value bytes or
None for a missing key exactly like ``txn.get(key.encode('ascii'))``.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Dict, List, Optional, Union

from .._lib import host_call, lib


class LmdbBackend:
    """LmdbBackend(db_paths, client_keys='default', readonly=True, lock=False, readahead=False) — read-only."""

    def __init__(self, db_paths, client_keys="default", readonly=True, lock=False, readahead=False, **kwargs):
        if isinstance(client_keys, str):
            client_keys = [client_keys]
        if isinstance(db_paths, (list, tuple)):
            self.db_paths = [str(v) for v in db_paths]
        else:
            self.db_paths = [str(db_paths)]
        assert len(client_keys) == len(self.db_paths), (
            "client_keys and db_paths should have the same length, "
            f"but received {len(client_keys)} and {len(self.db_paths)}.")
        if not readonly:
            raise ValueError("LmdbBackend: this build reads LMDB environments read-only")
        self._client: Dict[str, int] = {}
        for client, path in zip(client_keys, self.db_paths):
            self._client[client] = host_call("lmdb_open", os.fsencode(path))

    def get(self, filepath, client_key) -> Optional[bytes]:
        filepath = str(filepath)
        assert client_key in self._client, f"client_key {client_key} is not in lmdb clients."
        key = filepath.encode("ascii")
        val, vlen = ctypes.c_void_p(), ctypes.c_long()
        host_call("lmdb_get", self._client[client_key], key, len(key), ctypes.byref(val), ctypes.byref(vlen))
        if vlen.value < 0:
            return None
        return ctypes.string_at(val.value, vlen.value)

    def entries(self, client_key) -> int:
        n, ps = ctypes.c_long(), ctypes.c_long()
        host_call("lmdb_stat", self._client[client_key], ctypes.byref(n), ctypes.byref(ps))
        return int(n.value)

    def close(self):
        for h in self._client.values():
            host_call("lmdb_close", h)
        self._client = {}

    def get_text(self, filepath):
        raise NotImplementedError


class HardDiskBackend:
    def get(self, filepath) -> bytes:
        with open(str(filepath), "rb") as f:
            return f.read()

    def get_text(self, filepath) -> str:
        with open(str(filepath), "r") as f:
            return f.read()


class FileClient:
    """FileClient(backend='disk' | 'lmdb', **kwargs).get(filepath, client_key='default')."""

    _backends = {"disk": HardDiskBackend, "lmdb": LmdbBackend}

    def __init__(self, backend="disk", **kwargs):
        if backend not in self._backends:
            raise ValueError(f"Backend {backend} is not supported. Currently supported ones"
                             f" are {list(self._backends.keys())}")
        self.backend = backend
        self.client = self._backends[backend](**kwargs)

    def get(self, filepath, client_key="default"):
        if self.backend == "lmdb":
            return self.client.get(filepath, client_key)
        return self.client.get(filepath)

    def get_text(self, filepath):
        return self.client.get_text(filepath)


def expand_with_sid_root(path_value: Optional[Union[str, os.PathLike]]) -> Optional[Path]:
    """basicsr/utils/sid_paths.py:86-104: env vars and '~' expanded, backslashes -> '/', absolute paths kept,
    relative ones resolved against $SID_ROOT (or $LOWLIGHT_ROOT), else the working directory.  (The reference also
    probes a list of candidate directories for SID_* markers; this build takes the root from the environment.)"""
    if path_value is None or path_value == "":
        return None
    text = os.fspath(path_value)
    raw = Path(os.path.expandvars(text).replace("\\", "/")).expanduser()
    if raw.is_absolute():
        return raw
    root = os.environ.get("SID_ROOT") or os.environ.get("LOWLIGHT_ROOT")
    base = Path(os.path.expandvars(root)).expanduser() if root else Path.cwd()
    try:
        return (base / raw).resolve()
    except Exception:
        return base / raw


__all__: List[str] = ["FileClient", "LmdbBackend", "HardDiskBackend", "expand_with_sid_root", "lib"]
