"""Element diff of the LN NHWC kernels between two builds: `python scripts/ln_diff.py save OUT.pt` (under NBP_LIB=...)
writes the outputs; `python scripts/ln_diff.py cmp A.pt B.pt` reports differing elements and the max ulp distance."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_ln_bits import CASES, _key  # noqa: E402


def outputs(case):
    from lowlight_image_enhancement_amd._lib import call, query
    dev = torch.device("cuda:0")
    M, C, dt, res = case
    td = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[dt]
    gen = torch.Generator(device=dev).manual_seed(M * 3 + C + dt)
    x = (torch.randn(M, C, device=dev, generator=gen) * 2 + 0.3).to(td)
    w, b = torch.randn(C, device=dev, generator=gen), torch.randn(C, device=dev, generator=gen)
    n, st = torch.empty(M, C, device=dev, dtype=td), torch.empty(M, 2, device=dev)
    call("ln_fwd_nhwc", x, w, b, n, st, M, C, 1e-6, dt)
    dn = torch.randn(M, C, device=dev, generator=gen).to(td)
    dres = torch.randn(M, C, device=dev, generator=gen).to(td) if res else None
    dx = torch.empty(M, C, device=dev, dtype=td)
    slab = torch.full((2, query("ln_nhwc_grid", M, C, dt), C), float("nan"), device=dev)
    call("ln_bwd_nhwc", dn, x, st, w, dres, dx, slab[0], slab[1], M, C, dt)
    torch.cuda.synchronize()
    return [t.cpu() for t in (n, st, dx, slab)]


if sys.argv[1] == "save":
    torch.save({_key(c): outputs(c) for c in CASES}, sys.argv[2])
else:
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        for name, u, v in zip(("n", "stats", "dx", "slab"), a[k], b[k]):
            iv = torch.int16 if u.element_size() == 2 else torch.int32
            d = (u.view(iv).long() - v.view(iv).long()).abs()
            if int(d.max()):
                print(f"{k} {name}: {int((d > 0).sum())}/{d.numel()} differ, max {int(d.max())} ulp, "
                      f"max abs {float((u.float() - v.float()).abs().max()):.3g}")
    print("compared", len(a), "cases")
