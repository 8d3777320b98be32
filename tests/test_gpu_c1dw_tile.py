"""Levels 0 / 1 with the 2C-wide tape kept on chip (reference NAFNet_arch.py:59-68: conv1, conv2
(depthwise 3x3), SimpleGate, the SCA's pool, and their backward).

* nbp_c1dw_fwd_tile: t1 / t2 / g bitwise those of the two-launch path (nbp_gemm_bf16 conv1 + nbp_dw_sg_pool_fwd), the
  pool partials equal to float64 sums of the gate products (fp32 summation order differs);
* nbp_c1dw_bwd_tile: dt1 bitwise that of nbp_sca_sg_dw_bwd on the stored tape (t1 / t2 rebuilt from n1 on chip), the
  depthwise weight / bias gradients against float64;
* a network whose levels 0 / 1 take the tile path trains like the stored-tape path (16-bit rounding moved only by the
  pool's summation order), and the fp32 parity mode never takes it."""
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu

DT = {1: torch.bfloat16, 2: torch.float16}
SHAPES = [(2, 256, 256, 32), (3, 37, 70, 32), (2, 128, 128, 64), (1, 19, 45, 64), (1, 16, 16, 32)]


def _operands(dev, dt, B, H, W, C, seed):
    Ht = DT[dt]
    gen = torch.Generator(device=dev).manual_seed(seed)
    M = B * H * W
    n1 = torch.randn(M, C, device=dev, generator=gen).to(Ht)
    w1 = (torch.randn(2 * C, C, device=dev, generator=gen) / C ** 0.5).to(Ht)
    b1 = torch.randn(2 * C, device=dev, generator=gen) * 0.1
    wdw = torch.randn(2 * C, 9, device=dev, generator=gen) / 3
    bdw = torch.randn(2 * C, device=dev, generator=gen) * 0.1
    return n1, w1, b1, wdw, bdw


def _two_launch_fwd(dev, dt, B, H, W, C, n1, w1, b1, wdw, bdw):
    from lowlight_image_enhancement_amd._lib import call, query
    Ht, M = DT[dt], B * H * W
    t1r, t2r, gr = (torch.empty(M, n, device=dev, dtype=Ht) for n in (2 * C, 2 * C, C))
    call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1r, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1, None, None, None)
    rows = query("dw_fwd_slab_rows", B, H, W, C, dt)
    slab = torch.empty(B * rows * C, device=dev)
    call("dw_sg_pool_fwd", t1r, wdw, bdw, t2r, gr, slab, B, H, W, C, dt)
    return t1r, t2r, gr


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", SHAPES)
def test_fwd_tile_bitwise_equals_two_launches(dev, dt, B, H, W, C):
    from lowlight_image_enhancement_amd._lib import call, query
    assert query("c1dw_tile_supported", B, H, W, C, dt) == 1
    Ht, M = DT[dt], B * H * W
    n1, w1, b1, wdw, bdw = _operands(dev, dt, B, H, W, C, B + H + W + C + dt)
    t1r, t2r, gr = _two_launch_fwd(dev, dt, B, H, W, C, n1, w1, b1, wdw, bdw)
    rows = query("c1dw_tile_rows", H, W, C)
    # outputs pre-filled with NaN: every element must be written
    t1, t2, g = (torch.full((M, n), float("nan"), device=dev, dtype=Ht) for n in (2 * C, 2 * C, C))
    pool = torch.full((B * rows * C,), float("nan"), device=dev)
    call("c1dw_fwd_tile", n1, w1, b1, wdw, bdw, t1, t2, g, pool, B, H, W, C, dt)
    torch.cuda.synchronize()
    assert torch.equal(t1.view(torch.int16), t1r.view(torch.int16))
    assert torch.equal(t2.view(torch.int16), t2r.view(torch.int16))
    assert torch.equal(g.view(torch.int16), gr.view(torch.int16))
    # pool partials vs float64 sums of the fp32 gate products of the rounded t1
    t1d = t1r.double().view(B, H, W, 2 * C).permute(0, 3, 1, 2)
    t2d = Fn.conv2d(t1d, wdw.double().view(2 * C, 1, 3, 3), bdw.double(), padding=1, groups=2 * C)
    gd = (t2d[:, :C] * t2d[:, C:]).sum((2, 3))
    got = pool.double().view(B, rows, C).sum(1)
    torch.testing.assert_close(got, gd, rtol=1e-4, atol=1e-3 * (H * W) ** 0.5)
    # the production form (t1 / t2 not kept) writes the same g and pool
    g2 = torch.full((M, C), float("nan"), device=dev, dtype=Ht)
    pool2 = torch.full_like(pool, float("nan"))
    call("c1dw_fwd_tile", n1, w1, b1, wdw, bdw, None, None, g2, pool2, B, H, W, C, dt)
    torch.cuda.synchronize()
    assert torch.equal(g2.view(torch.int16), g.view(torch.int16)) and torch.equal(pool2, pool)


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", SHAPES)
def test_bwd_tile_dt1_bitwise_and_weight_grads(dev, dt, B, H, W, C):
    from lowlight_image_enhancement_amd._lib import call, query
    Ht, M = DT[dt], B * H * W
    n1, w1, b1, wdw, bdw = _operands(dev, dt, B, H, W, C, 7 * B + H + W + C + dt)
    t1r, t2r, _ = _two_launch_fwd(dev, dt, B, H, W, C, n1, w1, b1, wdw, bdw)
    gen = torch.Generator(device=dev).manual_seed(B * H + C)
    dh = torch.randn(M, C, device=dev, generator=gen).to(Ht)
    a = torch.rand(B, C, device=dev, generator=gen) + 0.5
    ds = torch.randn(B, C, device=dev, generator=gen) * 10
    # the stored-tape path
    dt1r = torch.empty(M, 2 * C, device=dev, dtype=Ht)
    dWr, dbr = torch.empty(2 * C * 9, device=dev), torch.empty(2 * C, device=dev)
    wsr = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
    call("sca_sg_dw_bwd", dh, a, ds, t2r, t1r, wdw, dt1r, dWr, dbr, wsr, B, H, W, C, dt)
    # the rebuilt-tape path
    dt1 = torch.full((M, 2 * C), float("nan"), device=dev, dtype=Ht)
    dW, db = torch.full_like(dWr, float("nan")), torch.full_like(dbr, float("nan"))
    ws = torch.empty(query("c1dw_bwd_workspace_floats", B, H, W, C), device=dev)
    call("c1dw_bwd_tile", dh, a, ds, n1, w1, b1, wdw, bdw, dt1, dW, db, ws, B, H, W, C, dt)
    torch.cuda.synchronize()
    assert torch.equal(dt1.view(torch.int16), dt1r.view(torch.int16))
    # weight / bias gradients vs float64 on the same rounded dt2 and t1
    dg = dh.double() * a.double().repeat_interleave(H * W, 0) + (ds.double() / (H * W)).repeat_interleave(H * W, 0)
    t2 = t2r.double()
    dt2 = torch.cat([(dg * t2[:, C:]).to(Ht).double(), (dg * t2[:, :C]).to(Ht).double()], 1)
    dt2n = dt2.view(B, H, W, 2 * C).permute(0, 3, 1, 2)
    t1n = t1r.double().view(B, H, W, 2 * C).permute(0, 3, 1, 2)
    t1p = Fn.pad(t1n, (1, 1, 1, 1))
    taps = [(dy, dx) for dy in range(3) for dx in range(3)]
    ref_w = torch.stack([(dt2n * t1p[:, :, dy:dy + H, dx:dx + W]).sum((0, 2, 3)) for dy, dx in taps], 1)
    abs_w = torch.stack([(dt2n * t1p[:, :, dy:dy + H, dx:dx + W]).abs().sum((0, 2, 3)) for dy, dx in taps], 1)
    # fp32 partial sums in any order: within 1e-5 of the sum of |terms| per element
    assert ((dW.view(2 * C, 9).double() - ref_w).abs() <= 1e-5 * abs_w + 1e-7).all()
    assert ((db.double() - dt2n.sum((0, 2, 3))).abs() <= 1e-5 * dt2n.abs().sum((0, 2, 3)) + 1e-7).all()
    assert ((dWr.view(2 * C, 9).double() - ref_w).abs() <= 1e-5 * abs_w + 1e-7).all()  # the stored-tape path too


def test_tile_shapes_not_served(dev):
    from lowlight_image_enhancement_amd._lib import NBPError, call, query
    assert query("c1dw_tile_supported", 1, 64, 64, 128, 2) == 0
    assert query("c1dw_tile_supported", 1, 256, 256, 32, 0) == 0
    assert query("c1dw_tile_supported", 1, 256, 256, 48, 1) == 0
    z = torch.zeros(8, device=dev)
    with pytest.raises(NBPError, match="unsupported shape"):
        call("c1dw_fwd_tile", z, z, z, z, z, None, None, z, z, 1, 64, 64, 128, 2)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B,H,W", [(2, 96, 80), (1, 1024, 1024)], ids=["96x80", "cfg5_1024"])
def test_tile_network_matches_stored_tape(dev, precision, B, H, W):
    """Width 32, two downs: levels 0 (C 32) and 1 (C 64) take the tile path.  Forward and parameter gradients against
    the stored-tape path of the same network within the 16-bit rounding that the pool's summation order can move --
    also at BASELINE configs[4]'s image size (1024^2: 1024 tiles per image at level 0, buffer offsets near 2^28 bytes;
    ADVICE r5)."""
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    torch.manual_seed(5)
    net = create_newbp_net(in_channels=3, width=32, enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1]).to(dev)
    net.precision = precision
    net.c1dw_tile_channels = (32, 64)
    assert net.tile_level(B, H, W, 32) and net.tile_level(B, H // 2, W // 2, 64)
    with torch.no_grad():
        net.flat.add_(torch.randn_like(net.flat) * 0.02)
    x = torch.rand(B, 3, H, W, device=dev)
    res = []
    for fuse in (True, False):
        net.fuse_c1dw_tile = fuse
        net.flat.grad = None
        out = net(x)
        out.square().mean().backward()
        res.append((out.detach().float().clone(), net.flat.grad.clone()))
    net.fuse_c1dw_tile = True
    (o1, g1), (o0, g0) = res
    assert (o1 - o0).abs().max().item() <= 2e-3 * (1 + o0.abs().max().item())
    assert (g1 - g0).norm().item() <= 2e-2 * g0.norm().item()
