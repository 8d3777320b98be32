"""Depthwise forward (dw 3x3 + SimpleGate + pool partials) at the level-0/1/2 shapes, graph-timed (env knobs such as
NBP_DW_FWD_TW apply).  Prints kernel us and the achieved rate on the algorithmic bytes (t1 2C in, t2 2C + g C out)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from micro_sca import timeit  # noqa: E402

dev = torch.device("cuda")
for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64), (16, 64, 64, 128), (16, 32, 32, 256), (16, 16, 16, 512)]:
    M = B * H * W
    t1 = torch.randn(M, 2 * C, device=dev).to(torch.bfloat16)
    w, b = torch.randn(2 * C, 9, device=dev), torch.randn(2 * C, device=dev)
    t2, g = torch.empty(M, 2 * C, device=dev, dtype=torch.bfloat16), torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    rows = query("dw_fwd_slab_rows", B, H, W, C, 1)
    pool = torch.empty(B * rows * C, device=dev)
    us = timeit(lambda: call("dw_sg_pool_fwd", t1, w, b, t2, g, pool, B, H, W, C, 1), 50)
    by = M * 5 * C * 2
    print(f"TW cap {os.environ.get('NBP_DW_FWD_TW', '-')}: B{B} {H}x{W} C{C}: {us:.1f} us, {by / us / 1e6:.2f} TB/s",
          flush=True)

# backward (fused SCA / SimpleGate / depthwise) at the same shapes
for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64), (16, 64, 64, 128), (16, 32, 32, 256), (16, 16, 16, 512)]:
    M = B * H * W
    t1, t2 = (torch.randn(M, 2 * C, device=dev).to(torch.bfloat16) for _ in range(2))
    dh = torch.randn(M, C, device=dev).to(torch.bfloat16)
    a, ds = torch.rand(B, C, device=dev), torch.randn(B, C, device=dev)
    w = torch.randn(2 * C, 9, device=dev)
    dt1 = torch.empty(M, 2 * C, device=dev, dtype=torch.bfloat16)
    dW, db = torch.empty(2 * C, 9, device=dev), torch.empty(2 * C, device=dev)
    ws = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
    us = timeit(lambda: call("sca_sg_dw_bwd", dh, a, ds, t2, t1, w, dt1, dW, db, ws, B, H, W, C, 1), 50)
    print(f"bwd TH {os.environ.get('NBP_DW_BWD_TH', '-')}: B{B} {H}x{W} C{C}: {us:.1f} us (incl. slab reductions)",
          flush=True)
