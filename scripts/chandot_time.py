"""Per-image channel dot (nbp_img_chan_dot, the SCA backward's da partials at levels 0/1) GPU time per launch
(HIP-graph replays) and algorithmic HBM rate at cfg2's levels 0/1 (B 16, fp16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64)]:
    M = B * H * W
    g = torch.Generator(device=dev).manual_seed(0)
    x, y = (torch.randn(M, C, device=dev, generator=g).half() for _ in range(2))
    slab = torch.empty(B, query("dw_chunks", B, H, W, C, 0), C, device=dev)
    t = timeit(lambda: call("img_chan_dot", x, y, slab, B, H, W, C, 2), reps=50)
    print(f"{H}x{W}xC{C}: {t:7.2f} us ({M * C * 4 / t / 1e3:5.0f} GB/s)", flush=True)
