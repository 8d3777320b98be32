"""Micro-benchmark: SCA forward / backward kernels at the NAFBlock level shapes (HIP events, 200 reps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lowlight_image_enhancement_amd._lib import call, query

dev = torch.device("cuda")


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for (B, H, W, C) in [(16, 256, 256, 32), (16, 32, 32, 256), (16, 16, 16, 512)]:
    rows = query("dw_fwd_slab_rows", B, H, W, C, 1)
    pool = torch.rand(B * rows * C, device=dev)
    wsca, bsca = torch.rand(C, C, device=dev), torch.rand(C, device=dev)
    mean, a = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
    tf = timeit(lambda: call("sca_fwd", pool, rows, wsca, bsca, mean, a, B, H * W, C))
    ch = query("dw_chunks", B, H, W, C, 0)
    da_slab = torch.rand(B * ch * C, device=dev)
    da, ds, dw, db = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev), torch.empty(C, C, device=dev), \
        torch.empty(C, device=dev)
    tb = timeit(lambda: call("sca_bwd", da_slab, ch, wsca, da, ds, B, C))
    x = torch.rand(B * H * W, C, device=dev, dtype=torch.bfloat16)
    ti = timeit(lambda: call("img_chan_dot", x, x, da_slab, B, H, W, C, 1))
    print(f"B{B} {H}x{W} C{C}: pool rows {rows}, da chunks {ch}: sca_fwd {tf:.1f} us, sca_bwd {tb:.1f} us, "
          f"img_chan_dot {ti:.1f} us", flush=True)
