"""The middle-level grouped weight-gradient launch alone: 6 NAFBlocks x {conv1 dW = dt1^T n1
[1024 x 512], conv3 U = dy^T (g (.) a) [512 x 512] with the per-image SCA scale, conv4 dW = dt4^T n2 [1024 x 512],
conv5 U = dout^T g2 [512 x 512]} at M = 16 x 16 x 16 = 4096, fp16, queued between nbp_wgrad_group(1) / (0) like the
executor's level backward, then the deferred slab reductions; REPS repetitions for PMC passes / timing:
    rocprofv3 --pmc <counters> --kernel-trace --stats -d <dir> -o run --output-format csv -- python scripts/wgroup_micro.py
WG_DT=1 for bf16; WG_BLOCKS / WG_C / WG_HW for other levels (e.g. WG_C=256 WG_HW=1024 WG_BLOCKS=5)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402

dev = torch.device("cuda:0")
dt = int(os.environ.get("WG_DT", "2"))
H = torch.float16 if dt == 2 else torch.bfloat16
C = int(os.environ.get("WG_C", "512"))
HW = int(os.environ.get("WG_HW", "256"))
NB = int(os.environ.get("WG_BLOCKS", "6"))
B = 16
M = B * HW
g = torch.Generator(device=dev).manual_seed(0)
R = lambda *s: torch.randn(*s, device=dev, generator=g).to(H)  # noqa: E731
probs = []
for _ in range(NB):
    for (n, k, scaled) in ((2 * C, C, False), (C, C, True), (2 * C, C, False), (C, C, False)):
        G, X = R(M, n), R(M, k)
        xs = torch.rand(B, k, device=dev, generator=g) if scaled else None
        dW = torch.empty(n, k, device=dev)
        n_ws = query("wgrad_workspace_floats", M, n, k)
        probs.append((G, X, xs, n, k, dW, torch.empty(n_ws, device=dev), n_ws))
reps = int(os.environ.get("REPS", "20"))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(reps + 2):
    if it == 2:
        e0.record()
    call("grad_reduce_defer")
    call("wgrad_group", 1)
    for G, X, xs, n, k, dW, ws, n_ws in probs:
        call("wgrad_f32", G, n, 0, X, k, 2 if xs is not None else 0, xs, HW, M, n, k, 0, 0, 0, 0, dW, None, ws, n_ws, dt)
    call("wgrad_group", 0)
    call("grad_reduce_flush", 1)
e1.record()
torch.cuda.synchronize()
fl = sum(2.0 * M * p[3] * p[4] for p in probs)
ms = e0.elapsed_time(e1) / reps
print(f"group of {len(probs)} problems (C {C}, M {M}): {ms * 1e3:.1f} us per group + reductions, "
      f"{fl / ms / 1e9:.1f} TFLOP/s incl. reductions")
