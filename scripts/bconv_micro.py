"""Image-boundary conv backward (nbp_intro_bwd / nbp_ending_bwd: weight-gradient slabs + their reductions, the ending
input gradient) at cfg2's level 0 (16 x 3 x 256 x 256, width 32, fp16 features), LDS-staged vs gather kernel, GPU
time per call from HIP-graph replays: python scripts/bconv_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
B, CI, H, W, Cf, dt = 16, 3, 256, 256, 32, 2
img, dy = torch.rand(B, CI, H, W, device=dev), torch.randn(B, CI, H, W, device=dev)
dout, feat = (torch.randn(B, H, W, Cf, device=dev).half() for _ in range(2))
w, we = torch.randn(Cf, CI, 3, 3, device=dev), torch.randn(CI, Cf, 3, 3, device=dev)
dw_i, db_i, dw_e, db_e = torch.empty_like(w), torch.empty(Cf, device=dev), torch.empty_like(we), torch.empty(CI, device=dev)
dfeat = torch.empty_like(feat)
ws = torch.empty(max(query("intro_bwd_workspace_floats", B, CI, H, W, Cf),
                     query("ending_bwd_workspace_floats", B, CI, H, W, Cf)), device=dev)
for gather in ("1", "0"):
    os.environ["NBP_BCONV_GATHER"] = gather
    ti = timeit(lambda: call("intro_bwd", img, dout, w, dw_i, db_i, None, ws, B, CI, H, W, H, W, Cf, dt))
    te = timeit(lambda: call("ending_bwd", dy, feat, we, dfeat, dw_e, db_e, ws, B, CI, H, W, H, W, Cf, dt))
    print(f"{'gather' if gather == '1' else 'lds   '}: intro_bwd {ti:6.1f} us, ending_bwd {te:6.1f} us", flush=True)
out, bias_i, bias_e = torch.empty_like(img), torch.randn(Cf, device=dev), torch.randn(CI, device=dev)
tf = timeit(lambda: call("intro_fwd", img, w, bias_i, dfeat, B, CI, H, W, H, W, Cf, dt))
te = timeit(lambda: call("ending_fwd", feat, we, bias_e, img, out, B, CI, H, W, H, W, Cf, dt))
print(f"intro_fwd {tf:6.1f} us, ending_fwd {te:6.1f} us", flush=True)
