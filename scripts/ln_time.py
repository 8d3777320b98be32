"""NHWC LayerNorm2d forward / backward GPU time per launch (HIP-graph replays) and algorithmic HBM rate at the cfg2
shapes (B 16, fp16) where the standalone kernels run (the middle level; levels 0-3 fuse LN into GEMM epilogues).
python scripts/ln_time.py [M,C ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
dt, td = 2, torch.float16
SHAPES = [(4096, 512), (16384, 256), (65536, 128)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for (M, C) in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    x, dn, dres = (torch.randn(M, C, device=dev, generator=g).to(td) for _ in range(3))
    w, b = torch.randn(C, device=dev, generator=g), torch.randn(C, device=dev, generator=g)
    n, st, dx = torch.empty_like(x), torch.empty(M, 2, device=dev), torch.empty_like(x)
    slab = torch.empty(2, query("ln_nhwc_grid", M, C, dt), C, device=dev)
    tf = timeit(lambda: call("ln_fwd_nhwc", x, w, b, n, st, M, C, 1e-6, dt), reps=100)
    tb = timeit(lambda: call("ln_bwd_nhwc", dn, x, st, w, dres, dx, slab[0], slab[1], M, C, dt), reps=100)
    bf, bb = M * C * 4 + M * 8, M * C * 8 + M * 8  # fwd x in, n out; bwd dn + x + dres in, dx out
    print(f"M{M} C{C}: fwd {tf:6.2f} us ({bf / tf / 1e3:5.0f} GB/s) | bwd {tb:6.2f} us ({bb / tb / 1e3:5.0f} GB/s)",
          flush=True)
