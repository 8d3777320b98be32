"""Micro-benchmark: conv3/conv5 skinny GEMM + standalone ln_fwd vs the fused nbp_gemm_res_ln at the level-0/1
shapes (graph-replayed, kernel time per call)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lowlight_image_enhancement_amd._lib import call
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from micro_sca import timeit  # noqa: E402  (graph-replay timer)

dev = torch.device("cuda")
for (M, N, amode) in [(16 * 256 * 256, 32, 2), (16 * 256 * 256, 32, 0), (16 * 128 * 128, 64, 2), (16 * 128 * 128, 64, 0)]:
    K = N
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    rows = M // 16
    scale = torch.rand(16, K, device=dev) + 0.5 if amode == 2 else None
    bias, rs = torch.randn(N, device=dev), torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev).to(torch.bfloat16)
    lnw, lnb = torch.randn(N, device=dev), torch.randn(N, device=dev)
    y, n, st = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev,
                                                                                 dtype=torch.bfloat16), torch.empty(M, 2, device=dev)
    t_g = timeit(lambda: call("gemm_bf16", A, K, amode, scale, rows, 1, W, K, y, N, 0, 1, M, N, K, 0, 0, 0, bias, R, rs,
                              None), 50)
    t_l = timeit(lambda: call("ln_fwd_nhwc", y, lnw, lnb, n, st, M, N, 1e-6, 1), 50)
    t_f = timeit(lambda: call("gemm_res_ln", A, K, amode, scale, rows, W, K, y, M, N, K, bias, R, rs, lnw, lnb, n, st,
                              1e-6, 1), 50)
    print(f"M={M} N={N} amode={amode}: gemm {t_g:.1f} + ln {t_l:.1f} = {t_g + t_l:.1f} us | fused {t_f:.1f} us",
          flush=True)
