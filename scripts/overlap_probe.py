"""Upside of running a deep level as two half-batch chains on two graph branches: a chain of L dependent GEMMs
(M x 512 x 512, each output the next input; the middle level's conv shapes at bs 16: M = 4096) on one stream vs two
M/2 chains on two streams forked / joined inside one captured graph.  GPU time per replay.
    python scripts/overlap_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402


def gemm(A, W, C, M, N, K):
    call("gemm_bf16", A, K, 0, None, 256, 2, W, K, C, N, 0, 2, M, N, K, 0, 0, 0, None, None, None, None)


def timed(g, iters=50):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda:0")
    L = 12
    for M, C in ((4096, 512), (16384, 256)):
        W = [(torch.randn(C, C, device=dev) / C ** 0.5).half() for _ in range(L)]
        bufs = [torch.randn(M, C, device=dev).half() for _ in range(L + 1)]

        def chain(lo, hi):
            for i in range(L):
                gemm(bufs[i][lo:hi], W[i], bufs[i + 1][lo:hi], hi - lo, C, C)

        s0 = torch.cuda.Stream()
        s1 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            chain(0, M)
        torch.cuda.current_stream().wait_stream(s0)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, stream=s0):
            chain(0, M)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s0):
            s1.wait_stream(s0)
            with torch.cuda.stream(s1):
                chain(M // 2, M)
            chain(0, M // 2)
            s0.wait_stream(s1)
        g3 = torch.cuda.CUDAGraph()  # the same halves one after the other on one stream
        with torch.cuda.graph(g3, stream=s0):
            chain(0, M // 2)
            chain(M // 2, M)
        for rep in range(2):
            t1, t2, t3 = timed(g1), timed(g2), timed(g3)
            print(f"M={M} C={C} chain of {L}: one stream {t1:7.1f} us ({t1 / L:5.2f}/GEMM) | two half chains on two "
                  f"branches {t2:7.1f} us ({t2 / L:5.2f}/pair) | the halves serial {t3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
