"""Narrow 16-bit weight gradients (nbp_wgrad_f32) on level-0/1 shapes: float64 check, per-call time (HIP events, 20
reps, slab reduction included) and the results saved for a bitwise comparison between two builds or env settings
(an env switch is read once per process; round 5 used it for the register-ring variants, profiles/r05_wgrad_ring/):
  NBP_LIB=a.so python scripts/wgrad_ring_check.py a.pt && NBP_LIB=b.so python scripts/wgrad_ring_check.py b.pt
  python scripts/wgrad_ring_check.py --compare a.pt b.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

# (M, N, K, x_mode, rows_per_img): level-1 conv1 / conv4 (128 x 64), U5 (64 x 64), level-0 / 1 U3 (per-image scale),
# ragged M
SHAPES = [(131072, 128, 64, 0, 0), (131072, 64, 64, 0, 0), (524288, 32, 32, 2, 65536), (131072, 64, 64, 2, 16384),
          (5 * 64 + 7, 128, 64, 0, 0), (3 * 4096, 32, 32, 2, 4096), (524288, 64, 32, 0, 0), (131072, 32, 64, 0, 0),
          (3 * 4096 + 640 + 5, 64, 32, 0, 0), (2 * 8192, 128, 32, 0, 0)]


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
        ok = True
        for k in a:
            eq = torch.equal(a[k], b[k])
            ok &= eq
            print(k, "bitwise" if eq else f"DIFF max {(a[k] - b[k]).abs().max().item():.3e}")
        sys.exit(0 if ok else 1)
    from lowlight_image_enhancement_amd._lib import call, query
    dev = torch.device("cuda:0")
    out = {}
    for M, N, K, xm, rows in SHAPES:
        gen = torch.Generator(device=dev).manual_seed(M + N + K)
        G = torch.randn(M, N, device=dev, generator=gen).to(torch.bfloat16)
        X = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
        sc = torch.rand(max(M // max(rows, 1), 1) * K, device=dev, generator=gen) if xm == 2 else None
        dW, db = torch.empty(N * K, device=dev), torch.empty(N, device=dev)
        nw = query("wgrad_workspace_floats", M, N, K)
        ws = torch.empty(nw, device=dev)
        args = (G, N, 0, X, K, xm, sc, rows if xm == 2 else 1, M, N, K, 0, 0, 0, 0, dW, db, ws, nw, 1)
        call("wgrad_f32", *args)
        torch.cuda.synchronize()
        ref = G.double().t() @ (X.double() * (sc.view(-1, K).repeat_interleave(rows, 0)[:M].double()
                                              if sc is not None else 1.0))
        err = (dW.view(N, K).double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call("wgrad_f32", *args)
        e1.record()
        torch.cuda.synchronize()
        key = f"M{M}_N{N}_K{K}_x{xm}"
        print(f"{key}: rel err vs f64 {err:.2e}, {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call (+ slab reduce)")
        assert err < 1e-4, key
        out[key + "_dW"], out[key + "_db"] = dW.cpu(), db.cpu()
    # space-to-depth gathers (the level-0 / 1 down conv: X gathered, N 64 x K 128; up conv: G gathered, N 128 x K 64)
    for B, gh, gw, cs, side in ((2, 64, 64, 32, "x"), (2, 64, 64, 32, "g"), (1, 9, 7, 32, "x"), (1, 9, 7, 32, "g")):
        M = B * gh * gw
        gen = torch.Generator(device=dev).manual_seed(M + cs + (side == "g"))
        fmap = torch.randn(B, 2 * gh, 2 * gw, cs, device=dev, generator=gen).to(torch.bfloat16)
        flat = fmap.view(B, gh, 2, gw, 2, cs).permute(0, 1, 3, 2, 4, 5).reshape(M, 4 * cs)  # k = (kh*2 + kw)*cs + c
        other = torch.randn(M, 2 * cs if side == "x" else 2 * cs, device=dev, generator=gen).to(torch.bfloat16)
        if side == "x":  # G plain [M][N = 2cs], X gathered (K = 4cs)
            N, K, G, X, gm, xm, csg, csx = 2 * cs, 4 * cs, other, fmap, 0, 1, 0, cs
            ref = other.double().t() @ flat.double()
        else:  # G gathered (N = 4cs), X plain [M][K = 2cs]
            N, K, G, X, gm, xm, csg, csx = 4 * cs, 2 * cs, fmap, other, 1, 0, cs, 0
            ref = flat.double().t() @ other.double()
        dW, db = torch.empty(N * K, device=dev), torch.empty(N, device=dev)
        nw = query("wgrad_workspace_floats", M, N, K)
        args = (G, N, gm, X, K, xm, None, 1, M, N, K, gh, gw, csg, csx, dW, db, torch.empty(nw, device=dev), nw, 1)
        call("wgrad_f32", *args)
        torch.cuda.synchronize()
        err = (dW.view(N, K).double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        bref = (other if side == "x" else flat).double().sum(0)
        berr = (db.double() - bref).abs().max().item() / (bref.abs().max().item() + 1e-12)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call("wgrad_f32", *args)
        e1.record()
        torch.cuda.synchronize()
        key = f"s2d_{side}_M{M}_N{N}_K{K}"
        print(f"{key}: rel err vs f64 {err:.2e} (db {berr:.2e}), {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call")
        assert err < 1e-4 and berr < 1e-4, key
        out[key + "_dW"], out[key + "_db"] = dW.cpu(), db.cpu()
    torch.save(out, sys.argv[1])


if __name__ == "__main__":
    main()
