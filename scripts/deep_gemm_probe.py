"""The deep-level 1x1-conv GEMM shapes (16x16 x C512 and 32x32 x C256 levels at bs 16: M = 4096 / 16384) on the
16-bit DMA GEMM, GPU time per launch (HIP-graph replays).  Run once per NBP_GLDS value to compare the
tile forms: python scripts/deep_gemm_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
TD = torch.float16
tot = 0.0
out = [f"NBP_GLDS={os.environ.get('NBP_GLDS', '-')}"]
for M, C in ((4096, 512), (16384, 256)):
    for N, K in ((2 * C, C), (C, C), (C, 2 * C)):
        A = torch.randn(M, K, device=dev).to(TD)
        W = (torch.randn(N, K, device=dev) / K ** 0.5).to(TD)
        Cm = torch.empty(M, N, device=dev, dtype=TD)
        us = timeit(lambda: call("gemm_bf16", A, K, 0, None, 256, 2, W, K, Cm, N, 0, 2, M, N, K, 0, 0, 0, None, None,
                                 None, None))
        tot += us
        out.append(f"M={M:5d} N={N:4d} K={K:4d}: {us:6.2f} us {2 * M * N * K / us / 1e6:6.1f} TF")
out.append(f"sum {tot:.2f} us")
print("\n".join(out), flush=True)
