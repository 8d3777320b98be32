"""SSIM loss forward / backward (nbp_ssim_loss_fwd / _bwd) at the cfg2 loss head (16 x 3 x 256 x 256, fp32), GPU time
per launch pair from HIP-graph replays: python scripts/ssim_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
N, C, H, W = 16, 3, 256, 256
x, y = torch.rand(N, C, H, W, device=dev), torch.rand(N, C, H, W, device=dev)
n = N * C * H * W
ws = torch.empty(query("ssim_workspace_floats", n), device=dev)
loss, up, gx = torch.empty(1, device=dev), torch.ones(1, device=dev), torch.empty_like(x)
f = timeit(lambda: call("ssim_loss_fwd", x, y, N, C, H, W, 11, 1.0, 1, 1, 0, ws, loss, None))
b = timeit(lambda: call("ssim_loss_bwd", x, y, N, C, H, W, 1, up, None, ws, gx))
print(f"ssim fwd {f:6.1f} us, bwd {b:6.1f} us  ({n * 4 * 5 / f / 1e3:.0f} / {n * 4 * 6 / b / 1e3:.0f} GB/s)", flush=True)
