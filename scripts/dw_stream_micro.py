"""The SCA + SimpleGate + depthwise backward per cfg2 level (bs 16, fp16): the staged-tile kernel (NBP_DW_STREAM=0)
vs the row-streaming one, HIP-graph replays (each graph captures 10 launches incl. the slab reductions), interleaved
rounds in one process; bytes = dh C + t2 2C + t1 2C in, dt1 2C out per pixel.
    python scripts/dw_stream_micro.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402
from scripts.c1dw_tile_micro import graph_time  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64), (16, 64, 64, 128), (16, 32, 32, 256)]:
        M = B * H * W
        g = torch.Generator(device=dev).manual_seed(0)
        dh = torch.randn(M, C, device=dev, generator=g).half()
        t1 = torch.randn(M, 2 * C, device=dev, generator=g).half()
        t2 = torch.randn(M, 2 * C, device=dev, generator=g).half()
        a = torch.rand(B, C, device=dev, generator=g) + 0.5
        ds = torch.randn(B, C, device=dev, generator=g)
        w = torch.randn(2 * C, 9, device=dev, generator=g) / 3
        dt1 = torch.empty(M, 2 * C, device=dev, dtype=torch.half)
        dW, db = torch.empty(2 * C * 9, device=dev), torch.empty(2 * C, device=dev)
        ws = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)

        def run():
            call("sca_sg_dw_bwd", dh, a, ds, t2, t1, w, dt1, dW, db, ws, B, H, W, C, 2)
        res = {"staged": [], "stream": []}
        for _ in range(3):
            for k in res:
                os.environ["NBP_DW_STREAM"] = "1" if k == "stream" else "0"
                res[k].append(graph_time(run, iters))
        mb = M * C * 2 * 7 / 1e6
        print(f"B{B} {H}x{W} C{C} ({mb:.0f} MB): " + "  ".join(
            f"{k} {min(v):7.1f} us ({mb / min(v):.2f} TB/s)" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
