"""Depthwise-backward microbenchmark at the level-0 shape (B 16, 256 x 256, C 32, fp16; DW_DT=1 bf16) for PMC passes:
    rocprofv3 --pmc <counters> --kernel-trace --stats -d <dir> -o run --output-format csv -- python scripts/dw_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402

dev = torch.device("cuda:0")
B, H, W, C = 16, 256, 256, int(os.environ.get("DW_C", "32"))
DT = int(os.environ.get("DW_DT", "2"))  # 1 bf16, 2 fp16 (the headline mode)
TD = {1: torch.bfloat16, 2: torch.float16}[DT]
M = B * H * W
g = torch.Generator(device=dev).manual_seed(0)
t1 = torch.randn(M, 2 * C, device=dev, generator=g).to(TD)
t2 = torch.randn(M, 2 * C, device=dev, generator=g).to(TD)
dh = torch.randn(M, C, device=dev, generator=g).to(TD)
a = torch.rand(B, C, device=dev, generator=g)
ds = torch.randn(B, C, device=dev, generator=g)
wdw = torch.randn(2 * C, 9, device=dev, generator=g)
dt1 = torch.empty(M, 2 * C, device=dev, dtype=TD)
dW, db = torch.empty(2 * C, 9, device=dev), torch.empty(2 * C, device=dev)
ws = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
for _ in range(10):
    call("sca_sg_dw_bwd", dh, a, ds, t2, t1, wdw, dt1, dW, db, ws, B, H, W, C, DT)
torch.cuda.synchronize()
print("ok")
