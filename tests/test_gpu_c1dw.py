"""The middle level's conv1 -> depthwise 3x3 -> SimpleGate -> pool in one whole-image launch (nbp_c1_dw_sg_pool,
VERDICT r3 item 4; reference NAFNet_arch.py:59-68).  t1 / t2 / g must be bitwise those of the two-launch path
(nbp_gemm_bf16 conv1 + nbp_dw_sg_pool_fwd), the pool sums equal up to fp32 summation order, and a whole network that
reaches the served level must train the same with and without the fusion."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {1: torch.bfloat16, 2: torch.float16}


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("S,C,B", [(16, 512, 16), (16, 512, 3), (16, 512, 1)])
def test_c1dw_bitwise_equals_two_launches(dev, dt, S, C, B):
    from lowlight_image_enhancement_amd._lib import call, query
    assert query("c1dw_supported", S, S, C, dt) == 1
    H = DT[dt]
    gen = torch.Generator(device=dev).manual_seed(S + C + B + dt)
    M = B * S * S
    n1 = torch.randn(M, C, device=dev, generator=gen).to(H)
    w1 = (torch.randn(2 * C, C, device=dev, generator=gen) / C ** 0.5).to(H)
    b1 = torch.randn(2 * C, device=dev, generator=gen) * 0.1
    wdw = torch.randn(2 * C, 9, device=dev, generator=gen) / 3
    bdw = torch.randn(2 * C, device=dev, generator=gen) * 0.1
    # two launches
    t1r, t2r, gr = (torch.empty(M, n, device=dev, dtype=H) for n in (2 * C, 2 * C, C))
    call("gemm_bf16", n1, C, 0, None, 1, dt, w1, C, t1r, 2 * C, 0, dt, M, 2 * C, C, 0, 0, 0, b1, None, None, None)
    rows = query("dw_fwd_slab_rows", B, S, S, C, dt)
    slab = torch.empty(B * rows * C, device=dev)
    call("dw_sg_pool_fwd", t1r, wdw, bdw, t2r, gr, slab, B, S, S, C, dt)
    # one launch (outputs pre-filled with NaN: every element must be written)
    t1, t2, g = (torch.full((M, n), float("nan"), device=dev, dtype=H) for n in (2 * C, 2 * C, C))
    pool = torch.full((B * C,), float("nan"), device=dev)
    call("c1_dw_sg_pool", n1, w1, b1, wdw, bdw, t1, t2, g, pool, B, S, S, C, dt)
    torch.cuda.synchronize()
    assert torch.equal(t1.view(torch.int16), t1r.view(torch.int16))
    assert torch.equal(t2.view(torch.int16), t2r.view(torch.int16))
    assert torch.equal(g.view(torch.int16), gr.view(torch.int16))
    ref_pool = slab.view(B, rows, C).sum(1).reshape(-1)
    torch.testing.assert_close(pool, ref_pool, rtol=2e-5, atol=1e-4)
    # and against float64 on the stored t1 (the depthwise conv with zero padding, the gate products' sum)
    t1d = t1.double().view(B, S, S, 2 * C).permute(0, 3, 1, 2)
    t2d = torch.nn.functional.conv2d(t1d, wdw.double().view(2 * C, 1, 3, 3), bdw.double(), padding=1, groups=2 * C)
    gd = t2d[:, :C] * t2d[:, C:]
    torch.testing.assert_close(pool.double().view(B, C), gd.sum((2, 3)), rtol=1e-4, atol=1e-2)


def test_c1dw_shapes_not_served(dev):
    from lowlight_image_enhancement_amd._lib import NBPError, call, query
    assert query("c1dw_supported", 64, 64, 128, 2) == 0
    assert query("c1dw_supported", 32, 32, 256, 2) == 0
    assert query("c1dw_supported", 16, 16, 512, 0) == 0
    assert query("c1dw_supported", 16, 32, 512, 1) == 0
    z = torch.zeros(8, device=dev)
    with pytest.raises(NBPError, match="unsupported shape"):
        call("c1_dw_sg_pool", z, z, z, z, z, z, z, z, z, 1, 64, 64, 128, 2)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_c1dw_network_matches_unfused(dev, precision):
    """A network whose middle level runs at 16 x 16 x C 512 (width 64, three downs, 128^2 input): the fused forward /
    backward equals the two-launch path within the 16-bit rounding the pool order can move (the SCA scale feeds a
    rounded product)."""
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    torch.manual_seed(11)
    net = create_newbp_net(in_channels=3, width=64, enc_blk_nums=[1, 1, 1], middle_blk_num=2,
                           dec_blk_nums=[1, 1, 1]).to(dev)
    net.precision = precision
    with torch.no_grad():
        net.flat.add_(torch.randn_like(net.flat) * 0.02)
    x = torch.rand(2, 3, 128, 128, device=dev)
    res = []
    for fuse in (True, False):
        net.fuse_c1dw = fuse
        net.flat.grad = None
        out = net(x)
        out.square().mean().backward()
        res.append((out.detach().float().clone(), net.flat.grad.clone()))
    net.fuse_c1dw = True
    (o1, g1), (o0, g0) = res
    assert (o1 - o0).abs().max().item() <= 2e-3 * (1 + o0.abs().max().item())
    assert (g1 - g0).norm().item() <= 2e-2 * g0.norm().item()
