"""Image-boundary conv kernels at cfg2's level 0 (B 16, 256 x 256, 3 image channels), fp16 features: GPU time per
launch (HIP-graph replays) of nbp_intro_fwd / nbp_intro_bwd / nbp_ending_fwd / nbp_ending_bwd by feature width.
python scripts/bconv_time.py [Cf ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
B, CI, H, W = 16, 3, 256, 256
for Cf in [int(v) for v in sys.argv[1:]] or [16, 32, 64]:
    g = torch.Generator(device=dev).manual_seed(0)
    img = torch.rand(B, CI, H, W, device=dev, generator=g)
    feat = torch.randn(B, H, W, Cf, device=dev, generator=g).half()
    w, bias = torch.randn(Cf, CI, 3, 3, device=dev, generator=g), torch.randn(Cf, device=dev, generator=g)
    we, be = torch.randn(CI, Cf, 3, 3, device=dev, generator=g), torch.randn(CI, device=dev, generator=g)
    dw, db, dwe, dbe = torch.empty_like(w), torch.empty_like(bias), torch.empty_like(we), torch.empty_like(be)
    out, dfeat = torch.empty_like(feat), torch.empty_like(feat)
    y = torch.empty_like(img)
    ws = torch.empty(max(query("intro_bwd_workspace_floats", B, CI, H, W, Cf),
                         query("ending_bwd_workspace_floats", B, CI, H, W, Cf)), device=dev)
    t = [timeit(lambda: call("intro_fwd", img, w, bias, out, B, CI, H, W, H, W, Cf, 2), reps=50),
         timeit(lambda: call("intro_bwd", img, feat, w, dw, db, None, ws, B, CI, H, W, H, W, Cf, 2), reps=50),
         timeit(lambda: call("ending_fwd", feat, we, be, img, y, B, CI, H, W, H, W, Cf, 2), reps=50),
         timeit(lambda: call("ending_bwd", img, feat, we, dfeat, dwe, dbe, ws, B, CI, H, W, H, W, Cf, 2), reps=50)]
    print(f"Cf {Cf:3d}: intro fwd {t[0]:6.1f} us | intro bwd (wgrad + 2 reductions) {t[1]:6.1f} | ending fwd {t[2]:6.1f}"
          f" | ending bwd (dx + wgrad + 2 reductions) {t[3]:6.1f}", flush=True)
