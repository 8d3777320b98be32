"""Build the gfx950 HIP library in-tree: lowlight_image_enhancement_amd/_lib/liblowlight_nbp.so.

hipcc --offload-arch=gfx950 per translation unit (in parallel), then one shared link.  No CUDA, no hipify, no
dual paths: the sources are written for CDNA4 directly.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(OUT_DIR, "liblowlight_nbp.so")
ARCH = os.environ.get("NBP_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + os.path.join(ROOT, "include"),
          "-Wno-unused-result", "-mcode-object-version=5"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "nbp.h")]
    return any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def _compile(src, obj, verbose):
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {os.path.basename(src)}:\n{r.stderr[-6000:]}")
    return obj


def build_library(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    objdir = os.path.join(OUT_DIR, "obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = _sources()
    objs = [os.path.join(objdir, os.path.splitext(os.path.basename(s))[0] + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _stale(o, s)]
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(lambda so: _compile(so[0], so[1], verbose), todo))
    if todo or force or not os.path.exists(LIB):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-lz", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
