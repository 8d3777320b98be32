"""Where the time of a deep-level GEMM goes: sweep K (K-steps at a fixed tile count), M (tile count at fixed K) and the
tile-size threshold for the plain 16-bit MFMA GEMM, beside torch.mm and a large square GEMM (clock / peak sanity).
python scripts/gemm_probe.py  (GPU time per launch from HIP-graph replays, as scripts/gemm_micro.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
TD = torch.float16


def ours(M, N, K):
    A = torch.randn(M, K, device=dev).to(TD)
    W = torch.randn(N, K, device=dev).to(TD)
    C = torch.empty(M, N, device=dev, dtype=TD)
    return timeit(lambda: call("gemm_bf16", A, K, 0, None, 256, 2, W, K, C, N, 0, 2, M, N, K, 0, 0, 0, None, None,
                               None, None))


def ref(M, N, K):
    A = torch.randn(M, K, device=dev).to(TD)
    W = torch.randn(N, K, device=dev).to(TD)
    return timeit(lambda: torch.mm(A, W.t()))


out = []
for K in (64, 128, 256, 512, 1024, 2048):
    us = ours(4096, 1024, K)
    out.append(f"K sweep  M=4096 N=1024 K={K:5d}: {us:7.2f} us {2 * 4096 * 1024 * K / us / 1e6:7.1f} TF")
for M in (1024, 2048, 4096, 8192, 16384, 32768):
    us = ours(M, 1024, 512)
    out.append(f"M sweep  M={M:5d} N=1024 K=512: {us:7.2f} us {2 * M * 1024 * 512 / us / 1e6:7.1f} TF")
for (M, N, K) in [(8192, 8192, 8192), (4096, 1024, 512)]:
    out.append(f"torch.mm M={M} N={N} K={K}: {ref(M, N, K):.2f} us")
us = ours(8192, 8192, 8192)
out.append(f"ours     M=8192 N=8192 K=8192: {us:.2f} us {2 * 8192 ** 3 / us / 1e6:.1f} TF")
print(f"NBP_GEMM_MINBLK={os.environ.get('NBP_GEMM_MINBLK', '-')}")
print("\n".join(out))
