"""Levels 0 / 1 fused forward (nbp_c1_dw_sg_pool_fwd: conv1 -> depthwise 3x3 -> SimpleGate -> pool partials in one
launch) against the two-launch path it replaces (nbp_gemm_bf16 conv1 + nbp_dw_sg_pool_fwd), NAFNet_arch.py:60-66.
t2 and g must be bitwise those of the depthwise kernel applied to the fused kernel's own t1 (same FMA order); t1 is
bitwise the level-0 skinny conv1 (C = 32: same MFMA sequence and epilogue) and within one 16-bit rounding of the tiled
conv1 (C = 64) and of float64; the pool partials are summed over other tiles, so their per-image totals agree to fp32
rounding.  Ragged shapes cover the tile edges and the zero padding of the halo."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {1: torch.bfloat16, 2: torch.float16}


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", [(2, 64, 64, 32), (3, 37, 45, 32), (2, 32, 48, 64), (1, 19, 23, 64),
                                     (16, 256, 256, 32)])
def test_c1_dw_fused_matches_two_launches(dev, dt, B, H, W, C):
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(B * H + W + C + dt)
    M, td = B * H * W, DT[dt]
    n1 = torch.randn(M, C, device=dev, generator=gen).to(td)
    w1 = (torch.randn(2 * C, C, device=dev, generator=gen) / C ** 0.5).to(td)
    b1 = 0.1 * torch.randn(2 * C, device=dev, generator=gen)
    wdw = 0.3 * torch.randn(2 * C, 9, device=dev, generator=gen)
    bdw = 0.1 * torch.randn(2 * C, device=dev, generator=gen)
    # two launches
    t1 = torch.empty(M, 2 * C, device=dev, dtype=td)
    call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1, None, None, None)
    chunks = query("dw_fwd_slab_rows", B, H, W, C, dt)
    t2, g = torch.empty(M, 2 * C, device=dev, dtype=td), torch.empty(M, C, device=dev, dtype=td)
    pool = torch.empty(B * chunks * C, device=dev)
    call("dw_sg_pool_fwd", t1, wdw, bdw, t2, g, pool, B, H, W, C, dt)
    # fused
    rows = query("c1_dw_slab_rows", H, W, C, dt)
    assert rows > 0
    T1, T2 = torch.empty(M, 2 * C, device=dev, dtype=td), torch.empty(M, 2 * C, device=dev, dtype=td)
    G, P = torch.empty(M, C, device=dev, dtype=td), torch.empty(B * rows * C, device=dev)
    call("c1_dw_sg_pool_fwd", n1, w1, b1, wdw, bdw, T1, T2, G, P, B, H, W, C, dt)
    # the depthwise pass on the fused kernel's own t1
    t2b, gb, poolb = torch.empty_like(t2), torch.empty_like(g), torch.empty_like(pool)
    call("dw_sg_pool_fwd", T1, wdw, bdw, t2b, gb, poolb, B, H, W, C, dt)
    torch.cuda.synchronize()
    assert torch.equal(T2, t2b) and torch.equal(G, gb)
    ref = n1.double() @ w1.double().t() + b1.double()
    tol = (2.0 ** -7 if dt == 1 else 2.0 ** -10) * ref.abs().clamp_min(1.0)
    assert ((T1.double() - ref).abs() <= tol).all()
    if C == 32:
        assert torch.equal(T1, t1) and torch.equal(T2, t2) and torch.equal(G, g)
    else:
        assert ((T1.double() - t1.double()).abs() <= tol).all()
    # pool partials: per-image channel sums of the fp32 gate products (before the 16-bit store of g), other tiles
    pf = P.view(B, rows, C).double().sum(1)
    pu = poolb.view(B, chunks, C).double().sum(1)
    torch.testing.assert_close(pf, pu, rtol=1e-5, atol=1e-5 * (H * W) ** 0.5)


def test_c1_dw_unsupported_shapes():
    from lowlight_image_enhancement_amd._lib import query
    assert query("c1_dw_slab_rows", 64, 64, 128, 2) == 0
    assert query("c1_dw_slab_rows", 64, 64, 32, 0) == 0
    assert query("c1_dw_slab_rows", 64, 64, 32, 2) == 8 * 2
