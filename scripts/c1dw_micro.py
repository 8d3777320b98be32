"""Levels 0 / 1 forward: conv1 + depthwise/SimpleGate/pool as two launches vs nbp_c1_dw_sg_pool_fwd (one), GPU time
per launch (HIP-graph replays).  python scripts/c1dw_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
dt, td = 2, torch.float16
out = []
for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64)]:
    M = B * H * W
    n1 = torch.randn(M, C, device=dev).to(td)
    w1 = (torch.randn(2 * C, C, device=dev) / C ** 0.5).to(td)
    b1, wdw, bdw = torch.randn(2 * C, device=dev), torch.randn(2 * C, 9, device=dev), torch.randn(2 * C, device=dev)
    t1, t2 = torch.empty(M, 2 * C, device=dev, dtype=td), torch.empty(M, 2 * C, device=dev, dtype=td)
    g = torch.empty(M, C, device=dev, dtype=td)
    ch = query("dw_fwd_slab_rows", B, H, W, C, dt)
    pool = torch.empty(B * max(ch, 64) * C, device=dev)
    rows = query("c1_dw_slab_rows", H, W, C, dt)
    poolf = torch.empty(B * rows * C, device=dev)
    t_g = timeit(lambda: call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1,
                              None, None, None), reps=50)
    t_d = timeit(lambda: call("dw_sg_pool_fwd", t1, wdw, bdw, t2, g, pool, B, H, W, C, dt), reps=50)
    t_f = timeit(lambda: call("c1_dw_sg_pool_fwd", n1, w1, b1, wdw, bdw, t1, t2, g, poolf, B, H, W, C, dt), reps=50)
    byt = M * 2 * (C + 2 * C + 2 * C + C)  # n1 in, t1 / t2 / g out
    out.append(f"{H}x{W}xC{C}: conv1 {t_g:7.1f} us + dw {t_d:7.1f} us = {t_g + t_d:7.1f} | fused {t_f:7.1f} us "
               f"({byt / t_f / 1e3:6.0f} GB/s of n1 + t1 + t2 + g)")
    print(out[-1], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/c1dw_micro.txt", "w").write("\n".join(out) + "\n")
