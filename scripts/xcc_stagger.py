"""Does the per-XCC dispatch stagger (scripts/gemm_timeline.py: XCC k starts ~0.5 k us after XCC 0 on a launch from an
idle GPU) repeat at every dependent launch?  Sequence on one stream: GEMM (M 4096 N 1024 K 512, stamps per
workgroup) -> trivial stamp kernel (512 workgroups) -> trivial stamp kernel, eager and as a replayed HIP graph; per XCC:
the GEMM's last workgroup end, each trivial kernel's first / last workgroup start (us from the GEMM's first start).
    NBP_LIB=$PWD/lowlight_image_enhancement_amd/_lib/probe/liblowlight_nbp.so python scripts/xcc_stagger.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, lib  # noqa: E402
from scripts.gemm_timeline import WORDS, read  # noqa: E402


def main():
    dll = lib().dll
    dll.nbp_probe_stamp.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    M, N, K = 4096, 1024, 512
    A = torch.randn(M, K, device=dev).half()
    W = (torch.randn(N, K, device=dev) / K ** 0.5).half()
    Cm = torch.empty(M, N, device=dev, dtype=torch.half)

    def seq():
        call("gemm_bf16", A, K, 0, None, 256, 2, W, K, Cm, N, 0, 2, M, N, K, 0, 0, 0, None, None, None, None)
        st = torch.cuda.current_stream().cuda_stream
        dll.nbp_probe_stamp(4096, 512, ctypes.c_void_p(st))
        dll.nbp_probe_stamp(8192, 512, ctypes.c_void_p(st))

    def report(tag):
        s = read(dll).astype(np.int64)
        g = s[:512]
        t0 = g[:, 0].min()
        gx = g[:, 7] & 0xF
        lines = [tag]
        for x in range(8):
            sel = gx == x
            row = f"  XCC {x}: GEMM start {(g[sel, 0].min() - t0) * .01:6.2f} end {(g[sel, 5].max() - t0) * .01:6.2f}"
            for r0 in (4096, 8192):
                k = s[r0:r0 + 512]
                kx = k[:, 7] & 0xF
                ks = k[kx == x, 0]
                row += f" | next start {(ks.min() - t0) * .01:6.2f}..{(ks.max() - t0) * .01:6.2f}"
            lines.append(row)
        print("\n".join(lines), flush=True)

    for _ in range(3):
        seq()
    torch.cuda.synchronize()
    seq()
    torch.cuda.synchronize()
    report("eager")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        seq()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        seq()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    report("graph replay")


if __name__ == "__main__":
    main()
