"""The deep levels' conv1 -> depthwise -> SimpleGate -> pool: one whole-image launch (nbp_c1_dw_sg_pool) against the
two launches it replaces (conv1 GEMM + dw_sg_pool_tiled), GPU time per step from HIP-graph replays, fp16, bs 16
python scripts/c1dw_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
dt, H, B = 2, torch.float16, 16
for S, C in ((16, 512),):
    M = B * S * S
    n1 = torch.randn(M, C, device=dev).to(H)
    w1 = (torch.randn(2 * C, C, device=dev) / C ** 0.5).to(H)
    b1 = torch.randn(2 * C, device=dev) * 0.1
    wdw, bdw = torch.randn(2 * C, 9, device=dev) / 3, torch.randn(2 * C, device=dev) * 0.1
    t1, t2, g = (torch.empty(M, n, device=dev, dtype=H) for n in (2 * C, 2 * C, C))
    rows = query("dw_fwd_slab_rows", B, S, S, C, dt)
    slab, pool = torch.empty(B * rows * C, device=dev), torch.empty(B * C, device=dev)

    def two():
        call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1, None, None, None)
        call("dw_sg_pool_fwd", t1, wdw, bdw, t2, g, slab, B, S, S, C, dt)

    def one():
        call("c1_dw_sg_pool", n1, w1, b1, wdw, bdw, t1, t2, g, pool, B, S, S, C, dt)
    a, o = timeit(two), timeit(one)
    print(f"{S}x{S} C {C}: two launches {a:6.2f} us, one launch {o:6.2f} us", flush=True)
