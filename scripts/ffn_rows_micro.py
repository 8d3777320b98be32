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


if __name__ == "__main__":
    main()
