"""Micro-benchmark: SCA forward / backward kernels at the NAFBlock level shapes (HIP events, 200 reps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lowlight_image_enhancement_amd._lib import call, query

dev = torch.device("cuda")


def timeit(fn, reps=200):
    """Kernel time per call: `reps` calls captured in one HIP graph and replayed (no host dispatch in the timing)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64), (16, 64, 64, 128), (16, 32, 32, 256), (16, 16, 16, 512)]:
        rows = query("dw_fwd_slab_rows", B, H, W, C, 1)
        pool = torch.rand(B * rows * C, device=dev)
        wsca, bsca = torch.rand(C, C, device=dev), torch.rand(C, device=dev)
        mean, a = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
        tf = timeit(lambda: call("sca_fwd", pool, rows, wsca, bsca, mean, a, B, H * W, C))
        ch = query("dw_chunks", B, H, W, C, 0)
        da_slab = torch.rand(B * ch * C, device=dev)
        da, ds, dw, db = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev), torch.empty(C, C, device=dev), \
            torch.empty(C, device=dev)
        tb = timeit(lambda: call("sca_bwd_fused", da_slab, ch, wsca, mean, ds, dw, db, B, C))
        x = torch.rand(B * H * W, C, device=dev, dtype=torch.bfloat16)
        ti = timeit(lambda: call("img_chan_dot", x, x, da_slab, B, H, W, C, 1))
        print(f"B{B} {H}x{W} C{C}: pool rows {rows}, da chunks {ch}: sca_fwd {tf:.1f} us, sca_bwd_fused {tb:.1f} us, "
              f"img_chan_dot {ti:.1f} us", flush=True)


if __name__ == "__main__":
    main()
