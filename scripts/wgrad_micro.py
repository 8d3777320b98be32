"""Wide weight-gradient kernel (or, WG_KIND=gemm, the bf16 GEMM C = A W^T) alone at the middle-level shape (M 4096,
N 1024, K 512, bf16), 20 eager launches, for PMC passes: rocprofv3 --pmc <counters> --kernel-trace --stats -d <dir> -o run --output-format csv --
python scripts/wgrad_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402

dev = torch.device("cuda:0")
M, N, K = (int(v) for v in os.environ.get("WG_SHAPE", "4096,1024,512").split(","))
G = torch.randn(M, N, device=dev).to(torch.bfloat16)
X = torch.randn(M, K, device=dev).to(torch.bfloat16)
dW = torch.empty(N, K, device=dev)
n_ws = query("wgrad_workspace_floats", M, N, K)
ws = torch.empty(n_ws, device=dev)
Wb = torch.randn(N, K, device=dev).to(torch.bfloat16)
for _ in range(20):
    if os.environ.get("WG_KIND", "wgrad") == "gemm":
        call("gemm_bf16", X, K, 0, None, 1, 1, Wb, K, G, N, 0, 1, M, N, K, 0, 0, 0, None, None, None, None)
    else:
        call("wgrad_f32", G, N, 0, X, K, 0, None, 1, M, N, K, 0, 0, 0, 0, dW, None, ws, n_ws, 1)
torch.cuda.synchronize()
print("ok")
