"""ctypes binding of the C-ABI in include/nbp.h (liblowlight_nbp.so, gfx950).

The signatures are parsed from the header itself, so header and binding cannot drift.  There is NO fallback:
if the library is missing or a call fails, this module raises.  `import torch` happens first so that the
library's libamdhip64.so.7 dependency binds to the HIP runtime torch already loaded (same SONAME), i.e. the
streams torch hands out are valid in the library.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Dict, List, Tuple

import torch

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NBP_LIB") or os.path.join(PKG, "_lib", "liblowlight_nbp.so")  # NBP_LIB: A/B builds
HEADER = os.path.join(os.path.dirname(PKG), "include", "nbp.h")

_C_TYPES = {
    "int": ctypes.c_int,
    "long": ctypes.c_long,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
    "nbp_stream_t": ctypes.c_void_p,
}


class NBPError(RuntimeError):
    pass


def parse_header(path: str = HEADER) -> Dict[str, Tuple[str, List[str]]]:
    """Return {name: (restype, [argtype, ...])} for every nbp_* function the header declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    out = {}
    for m in re.finditer(r"(const char\*|int|size_t|void)\s+(nbp_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                if "*" in a:
                    types.append("ptr")
                else:
                    t = a.rsplit(" ", 1)[0].replace("const ", "")
                    types.append(t)
        out[name] = (ret, types)
    return out


class _Lib:
    def __init__(self):
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"HIP library not built: {LIB_PATH} is missing. Run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        self.dll = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        self.sigs = parse_header()
        for name, (ret, types) in self.sigs.items():
            fn = getattr(self.dll, name)  # AttributeError = header/library mismatch, loud by design
            fn.argtypes = [ctypes.c_void_p if t == "ptr" else _C_TYPES[t] for t in types]
            fn.restype = {"int": ctypes.c_int, "size_t": ctypes.c_size_t, "const char*": ctypes.c_char_p,
                          "void": None}[ret]
        if self.dll.nbp_version() != 1:
            raise ImportError("liblowlight_nbp.so version mismatch")

    def __getattr__(self, name):
        return getattr(self.dll, name)


_lib = None


def lib() -> _Lib:
    global _lib
    if _lib is None:
        _lib = _Lib()
    return _lib


def ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# Optional live profiler: {name: callback(args, start_event, end_event)} — bench.py times the launches of one
# kernel class with HIP events recorded on the stream the kernel is launched on (torch's current stream).
PROFILE: Dict[str, object] = {}


def call(name: str, *args) -> int:
    """Call nbp_<name>(..., stream) with tensors converted to device pointers; raise on a negative return."""
    if PROFILE and name in PROFILE:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = _call(name, args)
        e1.record()
        PROFILE[name](args, e0, e1)
        return rc
    return _call(name, args)


def _call(name: str, args) -> int:
    L = lib()
    fn = getattr(L.dll, "nbp_" + name)
    conv = []
    for a in args:
        if isinstance(a, torch.Tensor):
            conv.append(a.data_ptr())
        elif isinstance(a, bool):
            conv.append(int(a))
        else:
            conv.append(a)
    conv.append(stream())
    rc = fn(*conv)
    if rc != 0:
        msg = L.dll.nbp_last_error_string().decode()
        raise NBPError(f"nbp_{name} failed ({rc}): {msg}")
    return rc


def query(name: str, *args) -> int:
    """Call a size/geometry query (no stream argument)."""
    return int(getattr(lib().dll, "nbp_" + name)(*args))


def host_call(name: str, *args) -> int:
    """Call a host-only entry point nbp_<name>(...) (no stream: LMDB / PNG); raise on a negative return, else
    return the value (e.g. an LMDB handle)."""
    L = lib()
    rc = getattr(L.dll, "nbp_" + name)(*args)
    if rc < 0:
        raise NBPError(f"nbp_{name} failed ({rc}): {L.dll.nbp_last_error_string().decode()}")
    return rc


def last_call_stats(which: int, n: int = 6) -> List[float]:
    """nbp_last_call_stats: host-side record of this thread's last nbp_wgrad_f32 (0), nbp_grad_reduce_flush (1) or
    nbp_wgrad_group end (2) call -- what it queued / launched and its algorithmic bytes (include/nbp.h)."""
    buf = (ctypes.c_double * n)()
    rc = lib().dll.nbp_last_call_stats(which, ctypes.cast(buf, ctypes.c_void_p), n)
    if rc != 0:
        raise NBPError(f"nbp_last_call_stats failed ({rc}): {lib().dll.nbp_last_error_string().decode()}")
    return list(buf)


def launch_timing(on: bool) -> None:
    """nbp_launch_timing: bracket each launch of the multi-instance entries (grouped weight gradients, the gradient-
    reduction flush) with HIP events (bench.py's per-instance roofline); switching clears the record."""
    lib().dll.nbp_launch_timing(1 if on else 0)


def launch_timing_records() -> List[Tuple[str, float, float, float]]:
    """[(kernel instance, ms, algorithmic FLOPs, algorithmic bytes)] of the launches recorded since launch_timing(True)
    (waits for each launch's end event)."""
    L = lib().dll
    out = []
    name = ctypes.create_string_buffer(128)
    buf = (ctypes.c_double * 3)()
    for i in range(L.nbp_launch_timing_count()):
        rc = L.nbp_launch_timing_get(i, ctypes.cast(name, ctypes.c_void_p), 128, ctypes.cast(buf, ctypes.c_void_p))
        if rc != 0:
            raise NBPError(f"nbp_launch_timing_get failed ({rc}): {L.nbp_last_error_string().decode()}")
        out.append((name.value.decode(), buf[0], buf[1], buf[2]))
    return out


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise NBPError(f"expected a float32 tensor on the GPU, got {t.dtype} on {t.device}")
