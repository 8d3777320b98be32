"""VGG19 3x3 conv shapes of cfg3 (bs 8 x 512^2, fp16): GPU time per launch of nbp_conv3x3_bf16 (forward + bias + ReLU,
and the input-gradient pass with the ReLU mask) beside MIOpen's channels-last conv2d, in TFLOP/s.
python scripts/conv_micro.py [B] [S] [VARIANT ...]   (HIP-graph replays, as scripts/gemm_micro.py).
A variant is a comma-separated list of NAME=VALUE environment settings read per launch (NBP_CONV_TILE, NBP_CONV_MAP,
NBP_IM2COL_TAP); every variant's outputs are checked bitwise against the first variant's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402
from scripts.gemm_micro_util import timeit  # noqa: E402

dev = torch.device("cuda:0")
TD = torch.float16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = int(sys.argv[2]) if len(sys.argv) > 2 else 512
VARIANTS = sys.argv[3:] or [""]
KNOBS = ("NBP_CONV_TILE", "NBP_CONV_MAP", "NBP_IM2COL_TAP")
SHAPES = [(S, 64, 64), (S // 2, 128, 128), (S // 4, 256, 256), (S // 8, 512, 512), (S // 16, 512, 512)]


def set_variant(v):
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        os.environ[k] = val


out = []
for (h, cin, cout) in SHAPES:
    torch.manual_seed(0)
    x = torch.randn(B, h, h, cin, device=dev).to(TD)
    w = (torch.randn(cout, 9, cin, device=dev) / (9 * cin) ** 0.5).to(TD)
    bias = 0.1 * torch.randn(cout, device=dev)
    wt = w.reshape(cout, 9, cin).flip(1).permute(2, 1, 0).contiguous()
    flop = 2.0 * B * h * h * cin * cout * 9
    ref = None
    for v in VARIANTS:
        set_variant(v)
        y = torch.empty(B, h, h, cout, device=dev, dtype=TD)
        dx = torch.empty(B, h, h, cin, device=dev, dtype=TD)
        t_f = timeit(lambda: call("conv3x3_bf16", x, B, h, h, cin, w, cout, bias, 0, None, y, 1, 2), reps=20)
        t_b = timeit(lambda: call("conv3x3_bf16", y, B, h, h, cout, wt, cin, None, 2, x, dx, 1, 2), reps=20)
        torch.cuda.synchronize()
        same = ""
        if ref is None:
            ref = (y.clone(), dx.clone())
        else:
            same = " bitwise=" + str(bool(torch.equal(y, ref[0]) and torch.equal(dx, ref[1])))
        out.append(f"{h:4d}^2 {cin:3d}->{cout:3d} [{v or 'default'}]: fwd {t_f:8.1f} us {flop / t_f / 1e6:6.1f} TF | "
                   f"dgrad {t_b:8.1f} us {flop / t_b / 1e6:6.1f} TF{same}")
        print(out[-1], flush=True)
    set_variant("")
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wn = w.reshape(cout, 3, 3, cin).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    t_m = timeit(lambda: torch.nn.functional.conv2d(xn, wn, padding=1), reps=20)
    out.append(f"{h:4d}^2 {cin:3d}->{cout:3d} MIOpen fwd {t_m:8.1f} us {flop / t_m / 1e6:6.1f} TF")
    print(out[-1], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/conv_micro.txt", "w").write("\n".join(out) + "\n")
