"""Gradient-slab reductions of the cfg2 stage flushes (shapes from NBP_REDUCE_LOG: wgrad / depthwise / LayerNorm
slabs), one nbp_reduce_slab per shape, HIP-graph replays (10 launches per replay); run once per library (NBP_LIB) to
compare builds.   python scripts/reduce_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call  # noqa: E402
from scripts.c1dw_tile_micro import graph_time  # noqa: E402

SHAPES = [(1024, 2048), (2048, 576), (1024, 64), (1024, 32), (512, 8192), (512, 1152), (8, 524288), (32, 131072),
          (128, 32768), (2048, 1280), (512, 512), (16, 9216), (256, 256), (7, 32768)]


def main():
    dev = torch.device("cuda:0")
    tot = 0.0
    lines = [f"NBP_LIB={os.environ.get('NBP_LIB', 'in-tree')}"]
    for S, L in SHAPES:
        slab = torch.randn(S, L, device=dev)
        out = torch.empty(L, device=dev)
        us = graph_time(lambda: call("reduce_slab", slab, S, L, out), 20)
        tot += us
        lines.append(f"S={S:5d} L={L:7d} ({S * L * 4 / 1e6:6.2f} MB): {us:6.2f} us  {S * L * 4 / us / 1e6:5.2f} TB/s")
    lines.append(f"sum {tot:.1f} us")
    print("\n".join(lines), flush=True)


if __name__ == "__main__":
    main()
