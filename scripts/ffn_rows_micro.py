"""Micro-benchmark of the deep-level FFN half (nbp_ffn_rows_fwd) against the launches it replaces, at the cfg2 shapes
(bs 16: level 2 = 64^2 x C 128, level 3 = 32^2 x C 256, middle = 16^2 x C 512; fp16), HIP-graph replays.
    python scripts/ffn_rows_micro.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402
from test_gpu_ffn_rows import _fused, _operands, _reference  # noqa: E402
from c1dw_tile_micro import graph_time  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    dt = 2
    for C, hw in ((128, 4096), (256, 1024), (512, 256)):
        B = 16
        M = B * hw
        o = _operands(dev, dt, B, hw, C, 1)
        for nxt in (True, False):
            ref = _reference(dev, dt, M, C, hw, o, nxt)
            got = {k: (torch.empty_like(v) if v is not None else None) for k, v in ref.items()}

            def old():
                _reference(dev, dt, M, C, hw, o, nxt)

            def new():
                _fused(dev, dt, M, C, hw, o, nxt, got)
            res = {"old": [], "new": []}
            for _ in range(3):
                res["old"].append(graph_time(old, iters))
                res["new"].append(graph_time(new, iters))
            mb = (M * C * (9 if nxt else 8) + 4 * C * C) * 2 / 1e6
            print(f"C{C} {hw} px/img B{B} next_ln={nxt}: launches {min(res['old']):.1f} us, fused {min(res['new']):.1f} us "
                  f"({mb:.1f} MB algorithmic -> {mb / min(res['new']):.2f} TB/s)", flush=True)




def main_bwd(iters=20):
    """the backward chain (nbp_ffn_rows_bwd) against its launches at the same shapes"""
    from test_gpu_ffn_rows import _bwd_reference, _dgrad_ln_reference, to_frag, DT
    dev = torch.device("cuda:0")
    dt = 2
    Ht = DT[dt]
    for C, hw in ((128, 4096), (256, 1024), (512, 256)):
        B = 16
        M = B * hw
        g = torch.Generator(device=dev).manual_seed(2)
        R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
        y = R(M, C).to(Ht)
        o = dict(dout=R(M, C).to(Ht), t4=R(M, 2 * C).to(Ht), y=y, st2=torch.rand(M, 2, device=dev) + 0.5,
                 lnw2=1 + 0.1 * R(C), g=R(M, C).to(Ht), w5t=(R(C, C) / C ** 0.5).to(Ht),
                 w4t=(R(C, 2 * C) / C ** 0.5).to(Ht), w3t=(R(C, C) / C ** 0.5).to(Ht))
        f5, f4, f3 = to_frag(o["w5t"]), to_frag(o["w4t"]), to_frag(o["w3t"])
        nb = M // 32
        outs = [torch.empty(M, n, device=dev, dtype=Ht) for n in (2 * C, C, C)]
        slabs = [torch.empty(nb * C, device=dev) for _ in range(3)]

        # the pending conv1 input gradient of the following block (nbp_ffn_rows_bwd with dt1)
        q = dict(dt1=R(M, 2 * C).to(Ht), w1t=(R(C, 2 * C) / C ** 0.5).to(Ht), x1=R(M, C).to(Ht),
                 st1=torch.rand(M, 2, device=dev) + 0.5, lnw1=1 + 0.1 * R(C), dres1=R(M, C).to(Ht))
        f1 = to_frag(q["w1t"])
        dx1 = torch.empty(M, C, device=dev, dtype=Ht)
        slabs1 = [torch.empty(nb * C, device=dev) for _ in range(2)]

        def old():
            _bwd_reference(dev, dt, M, C, hw, o)

        def new():
            call("ffn_rows_bwd", o["dout"], o["t4"], o["y"], o["st2"], o["lnw2"], o["g"], f5, f4, f3, *outs, *slabs,
                 *(None,) * 9, M, C, hw, dt)

        def old_pre():
            _dgrad_ln_reference(dev, dt, M, C, q["dt1"], q["w1t"], q["x1"], q["st1"], q["lnw1"], q["dres1"])
            new()

        def new_pre():
            call("ffn_rows_bwd", None, o["t4"], o["y"], o["st2"], o["lnw2"], o["g"], f5, f4, f3, *outs, *slabs,
                 q["dt1"], f1, q["x1"], q["st1"], q["lnw1"], q["dres1"], dx1, *slabs1, M, C, hw, dt)
        res = {"old": [], "new": [], "old_pre": [], "new_pre": []}
        for _ in range(3):
            for k, f in (("old", old), ("new", new), ("old_pre", old_pre), ("new_pre", new_pre)):
                res[k].append(graph_time(f, iters))
        mb = (M * C * 9 + 4 * C * C) * 2 / 1e6
        print(f"bwd C{C} {hw} px/img B{B}: launches {min(res['old']):.1f} us, fused {min(res['new']):.1f} us "
              f"({mb:.1f} MB algorithmic -> {mb / min(res['new']):.2f} TB/s); + conv1 dgrad/norm1: launches + fused "
              f"{min(res['old_pre']):.1f} us, one launch {min(res['new_pre']):.1f} us", flush=True)


if __name__ == "__main__":
    main()
    main_bwd()
