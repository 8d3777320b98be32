"""Micro-benchmark of the level-0/1 tile kernels against the stored-tape launches they replace, at the cfg2 shapes
(bs 16: level 0 = 256^2 x C 32, level 1 = 128^2 x C 64, fp16), HIP-graph replays of each form:
  fwd old: conv1 (nbp_gemm_bf16) + nbp_dw_sg_pool_fwd (t1 / t2 / g written)
  fwd new: nbp_c1dw_fwd_tile (g + pool partials only)
  bwd old: nbp_sca_sg_dw_bwd (+ its slab reductions)
  bwd new: nbp_c1dw_bwd_tile (+ its slab reductions)
    python scripts/c1dw_tile_micro.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402


def graph_time(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * 10)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    dt, Ht = 2, torch.float16
    for (B, H, W, C) in [(16, 256, 256, 32), (16, 128, 128, 64)]:
        M = B * H * W
        g = torch.Generator(device=dev).manual_seed(0)
        n1 = torch.randn(M, C, device=dev, generator=g).to(Ht)
        w1 = (torch.randn(2 * C, C, device=dev, generator=g) / C ** 0.5).to(Ht)
        b1 = torch.randn(2 * C, device=dev, generator=g) * 0.1
        wdw = torch.randn(2 * C, 9, device=dev, generator=g) / 3
        bdw = torch.randn(2 * C, device=dev, generator=g) * 0.1
        t1, t2, gg = (torch.empty(M, n, device=dev, dtype=Ht) for n in (2 * C, 2 * C, C))
        rows = query("dw_fwd_slab_rows", B, H, W, C, dt)
        slab = torch.empty(B * rows * C, device=dev)
        rows_t = query("c1dw_tile_rows", H, W, C)
        pool = torch.empty(B * rows_t * C, device=dev)
        dh = torch.randn(M, C, device=dev, generator=g).to(Ht)
        a = torch.rand(B, C, device=dev, generator=g) + 0.5
        ds = torch.randn(B, C, device=dev, generator=g)
        dt1 = torch.empty(M, 2 * C, device=dev, dtype=Ht)
        dW, db = torch.empty(2 * C * 9, device=dev), torch.empty(2 * C, device=dev)
        ws_old = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
        ws_new = torch.empty(query("c1dw_bwd_workspace_floats", B, H, W, C), device=dev)

        def conv1():
            call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1, None, None, None)

        def dwf():
            call("dw_sg_pool_fwd", t1, wdw, bdw, t2, gg, slab, B, H, W, C, dt)

        def fwd_old():
            conv1()
            dwf()

        def fwd_new():
            call("c1dw_fwd_tile", n1, w1, b1, wdw, bdw, None, None, gg, pool, B, H, W, C, dt)

        def bwd_old():
            call("sca_sg_dw_bwd", dh, a, ds, t2, t1, wdw, dt1, dW, db, ws_old, B, H, W, C, dt)

        def bwd_new():
            call("c1dw_bwd_tile", dh, a, ds, n1, w1, b1, wdw, bdw, dt1, dW, db, ws_new, B, H, W, C, dt)

        fwd_old()
        res = {k: [] for k in ("conv1", "dw_fwd", "fwd_old", "fwd_new", "bwd_old", "bwd_new")}
        for _ in range(3):  # interleaved rounds in one process
            for k, fn in (("conv1", conv1), ("dw_fwd", dwf), ("fwd_old", fwd_old), ("fwd_new", fwd_new),
                          ("bwd_old", bwd_old), ("bwd_new", bwd_new)):
                res[k].append(graph_time(fn, iters))
        mb = M * C * 2 / 1e6
        print(f"B{B} {H}x{W} C{C} fp16 (M*C*2 = {mb:.1f} MB):", flush=True)
        for k, v in res.items():
            print(f"  {k:8s} {min(v):8.1f} us  (rounds: {', '.join(f'{x:.1f}' for x in v)})", flush=True)
        print(f"  fwd new algorithmic bytes n1 + g = {2 * mb:.1f} MB -> {2 * mb / min(res['fwd_new']):.2f} TB/s; "
              f"bwd new dh + n1 + dt1 = {4 * mb:.1f} MB -> {4 * mb / min(res['bwd_new']):.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
