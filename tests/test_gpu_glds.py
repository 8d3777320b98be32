"""The LDS-DMA (global_load_lds) tiled GEMM against the register-staged tiled GEMM: same tiles, same fragment order and
MFMA sequence, so every output must be bitwise identical (NBP_GLDS=0 selects the register-staged kernel, unset the
DMA ring with its depth chosen per launch; the knob is read per launch).  Covers every A mode the DMA path serves (plain, per-image scale,
space-to-depth gather, 3x3 im2col with zero padding), the C modes of the deep-level GEMMs, ragged M / N, a K tail
(K % 64 != 0), both 16-bit types, and the fused-LayerNorm entries.  Accuracy against float64 is covered by the
existing GEMM tests, which run on the DMA path by default."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def run_modes(fn, modes=("0", "auto")):
    outs = {}
    old = os.environ.get("NBP_GLDS")
    try:
        for ns in modes:  # auto (unset): the depth chosen per launch from the grid
            if ns == "auto":
                os.environ.pop("NBP_GLDS", None)
            else:
                os.environ["NBP_GLDS"] = ns
            outs[ns] = [t.clone() for t in fn()]
            torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("NBP_GLDS", None)
        else:
            os.environ["NBP_GLDS"] = old
    for ns in modes[1:]:
        for a, b in zip(outs[modes[0]], outs[ns]):
            assert torch.equal(a, b), f"NBP_GLDS={ns} differs from NBP_GLDS={modes[0]}"


DT = {1: torch.bfloat16, 2: torch.float16}


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("M,N,K", [(4096, 1024, 512), (4136, 1000, 520), (16384, 256, 256), (100, 136, 72),
                                   (4096, 512, 1024)])
def test_glds_plain_bias_residual(dev, dt, M, N, K):
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(M + N + K + dt)
    A = torch.randn(M, K, device=dev, generator=gen).to(DT[dt])
    W = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(DT[dt])
    bias, sc = torch.randn(N, device=dev, generator=gen), torch.randn(N, device=dev, generator=gen)
    R = torch.randn(M, N, device=dev, generator=gen).to(DT[dt])
    C0, C1 = torch.empty(M, N, device=dev, dtype=DT[dt]), torch.empty(M, N, device=dev)

    def fn():
        call("gemm_bf16", A, K, 0, None, 1, dt, W, K, C0, N, 0, dt, M, N, K, 0, 0, 0, bias, R, sc, None)
        call("gemm_bf16", A, K, 0, None, 1, dt, W, K, C1, N, 0, 0, M, N, K, 0, 0, 0, None, None, None, None)
        return C0, C1
    run_modes(fn)
    ref = A.double() @ W.double().t()
    assert (C1.double() - ref).abs().max().item() < 1e-3 * K ** 0.5


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("M,C,rows", [(4096, 512, 256), (16384, 256, 1024), (2048, 128, 128)])
def test_glds_scale_simplegate(dev, dt, M, C, rows):
    """conv4 with the SimpleGate epilogue and the SCA-scaled conv3 / conv5 dgrad with the SimpleGate adjoint."""
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(M + C + dt)
    A = torch.randn(M, C, device=dev, generator=gen).to(DT[dt])
    W = (torch.randn(2 * C, C, device=dev, generator=gen) / C ** 0.5).to(DT[dt])
    b = torch.randn(2 * C, device=dev, generator=gen)
    scale = torch.rand(M // rows, C, device=dev, generator=gen) + 0.5
    Wd = (torch.randn(C, C, device=dev, generator=gen) / C ** 0.5).to(DT[dt])
    t, g = torch.empty(M, 2 * C, device=dev, dtype=DT[dt]), torch.empty(M, C, device=dev, dtype=DT[dt])
    dtt, y = torch.empty(M, 2 * C, device=dev, dtype=DT[dt]), torch.empty(M, C, device=dev, dtype=DT[dt])

    def fn():
        call("gemm_bf16", A, C, 0, None, 1, dt, W, C, t, 2 * C, 4, dt, M, 2 * C, C, 0, 0, 0, b, None, None, g)
        call("gemm_bf16", A, C, 2, scale, rows, dt, Wd, C, dtt, 2 * C, 5, dt, M, C, C, 0, 0, 0, None, t, None, None)
        call("gemm_bf16", A, C, 2, scale, rows, dt, Wd, C, y, C, 0, dt, M, C, C, 0, 0, 0, b[:C].contiguous(), None,
             None, None)
        return t, g, dtt, y
    run_modes(fn)


@pytest.mark.parametrize("B,gh,gw,cs", [(16, 16, 16, 256), (2, 32, 24, 64), (3, 5, 7, 128)])
def test_glds_space_to_depth(dev, B, gh, gw, cs):
    """down conv (2x2 / stride 2 as a space-to-depth GEMM, K = 4 cs) and the up conv's depth-to-space epilogue."""
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(B * gh + cs)
    x = torch.randn(B, 2 * gh, 2 * gw, cs, device=dev, generator=gen).to(torch.bfloat16)
    M, K, N = B * gh * gw, 4 * cs, 2 * cs
    W = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=gen)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    Wu = (torch.randn(4 * cs, N, device=dev, generator=gen) / N ** 0.5).to(torch.bfloat16)
    up = torch.empty(B, 2 * gh, 2 * gw, cs, device=dev, dtype=torch.bfloat16)

    def fn():
        call("gemm_bf16", x, K, 1, None, 1, 1, W, K, y, N, 0, 1, M, N, K, gh, gw, cs, bias, None, None, None)
        call("gemm_bf16", y, N, 0, None, 1, 1, Wu, N, up, N, 1, 1, M, 4 * cs, N, gh, gw, cs, None, None, None, None)
        return y, up
    run_modes(fn)


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(1, 64, 64, 64, 128), (2, 17, 23, 128, 64), (1, 32, 32, 256, 256),
                                            (3, 130, 170, 64, 64), (4, 128, 128, 128, 128), (2, 96, 180, 64, 256),
                                            (4, 128, 128, 256, 256), (3, 100, 180, 64, 264)])
def test_glds_conv3x3(dev, B, H, W, Cin, Cout):
    """VGG 3x3 convolution (implicit GEMM, zero padding read from the zero page): bias + ReLU and the ReLU-mask form.
    The last two shapes (N >= 256, >= 256 workgroups) run the 256 x 256 tiles with the two-pass epilogue (ragged M and
    N in the last); the register-staged kernel (NBP_GLDS=0) keeps 128-row tiles and the plain tile order, so every
    tile shape, the per-stage tap of the DMA issue and the XCD-contiguous tile order are compared bitwise with it."""
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(B * H + Cin)
    x = torch.randn(B, H, W, Cin, device=dev, generator=gen).to(torch.bfloat16)
    w = (torch.randn(Cout, 9 * Cin, device=dev, generator=gen) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev, generator=gen)
    y, ym = (torch.empty(B, H, W, Cout, device=dev, dtype=torch.bfloat16) for _ in range(2))

    def fn():
        call("conv3x3_bf16", x, B, H, W, Cin, w, Cout, b, 0, None, y, 1, 1)
        call("conv3x3_bf16", x, B, H, W, Cin, w, Cout, None, 2, y, ym, 1, 1)
        return y, ym
    run_modes(fn)


@pytest.mark.parametrize("M,N,K,amode", [(4096, 256, 256, 2), (16384, 128, 256, 0), (333, 256, 512, 0),
                                          (4096, 512, 512, 2), (4096, 512, 1024, 0), (700, 512, 512, 0)])
def test_glds_fused_layernorm(dev, M, N, K, amode):
    """conv3 / conv5 with the LayerNorm forward in the epilogue, and the conv1 / conv4 dgrad with the LN backward."""
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(M + N + K)
    rows = 256 if amode == 2 else M
    A = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(torch.bfloat16)
    scale = torch.rand(M // rows, K, device=dev, generator=gen) + 0.5 if amode == 2 else None
    bias, rs = torch.randn(N, device=dev, generator=gen), torch.randn(N, device=dev, generator=gen)
    R = torch.randn(M, N, device=dev, generator=gen).to(torch.bfloat16)
    lnw, lnb = torch.randn(N, device=dev, generator=gen), torch.randn(N, device=dev, generator=gen)
    y, n, st = (torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev,
                dtype=torch.bfloat16), torch.empty(M, 2, device=dev))
    Wt = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(torch.bfloat16)
    dres = torch.randn(M, N, device=dev, generator=gen).to(torch.bfloat16)
    dx, dlnw, dlnb = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(N, device=dev), torch.empty(
        N, device=dev)
    n_ws = query("dgrad_ln_workspace_floats", M, N)
    ws = torch.empty(n_ws, device=dev)

    def fn():
        call("gemm_res_ln", A, K, amode, scale, rows, W, K, y, M, N, K, bias, R, rs, lnw, lnb, n, st, 1e-6, 1)
        call("dgrad_ln_bwd", A, K, Wt, K, M, N, K, y, st, lnw, dres, dx, dlnw, dlnb, ws, n_ws, 1)
        return y, n, st, dx, dlnw, dlnb
    # N = 512 (64 x 512 tiles) exists on the DMA path only (its register-staged double buffer exceeds the LDS):
    # accuracy vs float64 is test_gpu_parity's
    if N != 512:
        run_modes(fn)
    else:
        fn()


@pytest.mark.parametrize("B,HW,C", [(16, 256, 512), (3, 1024, 256)])
def test_glds_chandot(dev, B, HW, C):
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(B * HW + C)
    M = B * HW
    A = torch.randn(M, C, device=dev, generator=gen).to(torch.bfloat16)
    Wt = (torch.randn(C, C, device=dev, generator=gen) / C ** 0.5).to(torch.bfloat16)
    g = torch.randn(M, C, device=dev, generator=gen).to(torch.bfloat16)
    d = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    slab = torch.empty(B * (HW // 64) * C, device=dev)

    def fn():
        call("gemm_bf16", A, C, 0, None, HW, 1, Wt, C, d, C, 8, 1, M, C, C, 0, 0, 0, None, g, None, slab)
        return d, slab
    run_modes(fn)


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("M,N,K,rows", [(4096, 1024, 512, 256), (16384, 256, 512, 1024), (65536, 128, 256, 4096),
                                        (3000, 256, 128, 0), (4160, 512, 512, 0)])
def test_glds_wide_wgrad(dev, dt, M, N, K, rows):
    """Wide weight gradient (N, K multiples of 128) with LDS-DMA panels vs the register-staged tile: dW bitwise (same
    MFMA sequence and per-image scale fold), the bias column sums (MFMA against ones vs register sums: another
    order) within fp32 rounding.  rows > 0: the per-image SCA column scale of X."""
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(M + N + K + dt)
    G = torch.randn(M, N, device=dev, generator=gen).to(DT[dt])
    X = torch.randn(M, K, device=dev, generator=gen).to(DT[dt])
    sc = torch.rand(max(M // max(rows, 1), 1), K, device=dev, generator=gen) + 0.5 if rows else None
    n_ws = query("wgrad_workspace_floats", M, N, K)
    ws = torch.empty(n_ws, device=dev)
    res = {}
    old = os.environ.get("NBP_WGRAD_GLDS")
    try:
        for ns in ("0", "2", "3", "4"):
            os.environ["NBP_WGRAD_GLDS"] = ns
            dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
            call("wgrad_f32", G, N, 0, X, K, 2 if rows else 0, sc, rows if rows else 1, M, N, K, 0, 0, 0, 0, dW, db,
                 ws, n_ws, dt)
            torch.cuda.synchronize()
            res[ns] = (dW, db)
    finally:
        if old is None:
            os.environ.pop("NBP_WGRAD_GLDS", None)
        else:
            os.environ["NBP_WGRAD_GLDS"] = old
    for ns in ("2", "3", "4"):
        assert torch.equal(res[ns][0], res["0"][0]), ns
        torch.testing.assert_close(res[ns][1], res["0"][1], rtol=1e-5, atol=1e-4 * M ** 0.5)
    Xe = X.double() * (sc.double().repeat_interleave(rows, 0)[:M] if rows else 1.0)
    ref = G.double().t() @ Xe
    assert (res["2"][0].double() - ref).abs().max().item() <= 1e-4 * M ** 0.5
    assert (res["2"][1].double() - G.double().sum(0)).abs().max().item() <= 1e-4 * M ** 0.5


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("M,N,K,rows", [(262144, 128, 64, 0), (262144, 64, 64, 16384), (5000, 64, 32, 0),
                                        (262144, 64, 32, 65536)])
def test_narrow_wgrad_vs_float64(dev, dt, M, N, K, rows):
    """Narrow weight gradients (N or K <= 64: levels 0 / 1, 64-row stages) vs float64; rows > 0: the per-image SCA
    column scale folded per image."""
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(M + N + K + dt)
    G = torch.randn(M, N, device=dev, generator=gen).to(DT[dt])
    X = torch.randn(M, K, device=dev, generator=gen).to(DT[dt])
    sc = torch.rand(M // rows, K, device=dev, generator=gen) + 0.5 if rows else None
    n_ws = query("wgrad_workspace_floats", M, N, K)
    ws = torch.empty(n_ws, device=dev)
    dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    call("wgrad_f32", G, N, 0, X, K, 2 if rows else 0, sc, rows if rows else 1, M, N, K, 0, 0, 0, 0, dW, db, ws, n_ws,
         dt)
    Xe = X.double() * (sc.double().repeat_interleave(rows, 0)[:M] if rows else 1.0)
    assert (dW.double() - G.double().t() @ Xe).abs().max().item() <= 1e-4 * M ** 0.5
    assert (db.double() - G.double().sum(0)).abs().max().item() <= 1e-4 * M ** 0.5


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("C,HW", [(512, 256), (256, 1024), (128, 4096)])
def test_wgrad_group_variants_bitwise(dev, dt, C, HW):
    """The grouped wide weight gradients of one U-Net level (nbp_wgrad_group: conv1 / conv4 dW [2C x C], conv3 U with
    the per-image SCA scale and conv5 U [C x C], two blocks) on every tile variant -- the register-staged tile
    (NBP_WGRAD_GLDS=0), the 4-wave LDS-DMA rings (3, 4), the loader / consumer split (43, 44: waves 4..7 issue the
    DMA, 0..3 multiply) and the 256-column tiles of the plain problems (83: 8 compute + 4 loader waves) -- give bitwise
    equal dW at equal M-splits (the same MFMA sequence per element); the bias column sums within fp32 rounding; dW
    against float64 also under the default split policy."""
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(C + HW + dt)
    B = 16 if C == 512 else 4
    M = B * HW
    probs = []
    for _ in range(2):
        for (n, k, scaled, bias) in ((2 * C, C, False, True), (C, C, True, False), (2 * C, C, False, True),
                                     (C, C, False, False)):
            G = torch.randn(M, n, device=dev, generator=gen).to(DT[dt])
            X = torch.randn(M, k, device=dev, generator=gen).to(DT[dt])
            xs = torch.rand(B, k, device=dev, generator=gen) + 0.5 if scaled else None
            probs.append((G, X, xs, n, k, bias))
    res = {}
    old = {k: os.environ.get(k) for k in ("NBP_WGRAD_GLDS", "NBP_WGROUP_SPLITS")}
    # (variant, NBP_WGRAD_GLDS, forced splits): equal splits for the bitwise comparison, then the default split policy
    runs = [(v, v, "2") for v in ("0", "3", "4", "43", "44", "83")] + [("43auto", "43", None), ("83auto", "83", None)]
    try:
        for name, ns, splits in runs:
            os.environ["NBP_WGRAD_GLDS"] = ns
            if splits is None:
                os.environ.pop("NBP_WGROUP_SPLITS", None)
            else:
                os.environ["NBP_WGROUP_SPLITS"] = splits
            outs = []
            call("grad_reduce_defer")
            call("wgrad_group", 1)
            for G, X, xs, n, k, bias in probs:
                n_ws = query("wgrad_workspace_floats", M, n, k)
                dW, db = torch.empty(n, k, device=dev), (torch.empty(n, device=dev) if bias else None)
                ws = torch.empty(n_ws, device=dev)
                call("wgrad_f32", G, n, 0, X, k, 2 if xs is not None else 0, xs, HW, M, n, k, 0, 0, 0, 0, dW, db, ws,
                     n_ws, dt)
                outs.append((dW, db, ws))
            call("wgrad_group", 0)
            call("grad_reduce_flush", 1)
            torch.cuda.synchronize()
            res[name] = [(a, b) for a, b, _ in outs]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for ns in ("3", "4", "43", "44", "83"):
        for (a, ab), (r, rb) in zip(res[ns], res["0"]):
            assert torch.equal(a, r), ns
            if rb is not None:
                torch.testing.assert_close(ab, rb, rtol=1e-5, atol=1e-4 * M ** 0.5)
    for name in ("44", "43auto", "83auto"):
        for (G, X, xs, n, k, bias), (dW, db) in zip(probs, res[name]):
            Xe = X.double() * (xs.double().repeat_interleave(HW, 0) if xs is not None else 1.0)
            assert (dW.double() - G.double().t() @ Xe).abs().max().item() <= 1e-4 * M ** 0.5, name
            if bias:
                assert (db.double() - G.double().sum(0)).abs().max().item() <= 1e-4 * M ** 0.5, name


