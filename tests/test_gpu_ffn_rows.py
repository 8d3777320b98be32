"""The deep-level FFN half in one row-stationary launch (nbp_ffn_rows_fwd; NAFNet_arch.py:69-80 after the SCA, with the
next block's norm1, arch_util.py:264-275): every tensor it stores -- y, n2 and its statistics, t4, g2, out and the next
block's n1 and statistics -- bitwise equal to the launches it replaces (conv3 with the SCA scale + residual and norm2,
conv4 with the SimpleGate epilogue, conv5 + residual (+ norm1)), at C 128 / 256 / 512 in both 16-bit types and images
of 256 / 1024 / 4096 rows; and the backward chain (nbp_ffn_rows_bwd) likewise for
dt4 / dy / dh; a network whose levels 2 / 3 / middle take both trains like the unfused network."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {1: torch.bfloat16, 2: torch.float16}
AM_SCALE, AM_PLAIN, CM_PLAIN, CM_SG = 2, 0, 0, 4
EPS = 1e-6


def _bits(t):
    return t.view(torch.int16) if t.dtype in (torch.float16, torch.bfloat16) else t.view(torch.int32)


def _operands(dev, dt, B, hw, C, seed):
    Ht = DT[dt]
    gen = torch.Generator(device=dev).manual_seed(seed)
    M = B * hw
    R = lambda *s: torch.randn(*s, device=dev, generator=gen)  # noqa: E731
    ops = dict(
        g=R(M, C).to(Ht), a=torch.rand(B, C, device=dev, generator=gen) + 0.5, x=(R(M, C) * 2 + 0.3).to(Ht),
        w3=(R(C, C) / C ** 0.5).to(Ht), b3=R(C) * 0.1, beta=R(C) * 0.3, lnw2=1 + 0.1 * R(C), lnb2=0.1 * R(C),
        w4=(R(2 * C, C) / C ** 0.5).to(Ht), b4=R(2 * C) * 0.1, w5=(R(C, C) / C ** 0.5).to(Ht), b5=R(C) * 0.1,
        gamma=R(C) * 0.3, lnw1=1 + 0.1 * R(C), lnb1=0.1 * R(C))
    return ops


def to_frag(W):
    """[N][K] -> fragment order (include/nbp.h nbp_weights_frag): 1-KB blocks (32-row tile, 16-wide k-step), lane l =
    row (l & 31), k half (l >> 5)"""
    N, K = W.shape
    return W.reshape(N // 32, 32, K // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(-1)


def _fused(dev, dt, M, C, hw, o, nxt, got):
    from lowlight_image_enhancement_amd._lib import call
    if "f3" not in o:
        o["f3"], o["f4"], o["f5"] = to_frag(o["w3"]), to_frag(o["w4"]), to_frag(o["w5"])
    call("ffn_rows_fwd", o["g"], o["a"], hw, o["x"], o["f3"], o["b3"], o["beta"], o["lnw2"], o["lnb2"],
         o["f4"], o["b4"], o["f5"], o["b5"], o["gamma"], o["lnw1"] if nxt else None,
         o["lnb1"] if nxt else None, got["y"], got["n2"], got["st2"], got["t4"], got["g2"], got["out"], got["nn1"],
         got["nst1"], M, C, EPS, dt)


def _reference(dev, dt, M, C, hw, o, nxt):
    """the launches the executor issued before (nafnet.py _block_fwd: conv3 / norm2, conv4 CM_SG, conv5 / norm1)"""
    from lowlight_image_enhancement_amd._lib import call
    Ht = DT[dt]
    E = lambda n: torch.empty(M, n, device=dev, dtype=Ht)  # noqa: E731
    y, n2, g2, out = E(C), E(C), E(C), E(C)
    t4 = E(2 * C)
    st2 = torch.empty(M, 2, device=dev)
    nn1, nst1 = (E(C), torch.empty(M, 2, device=dev)) if nxt else (None, None)
    if C in (128, 256):
        call("gemm_res_ln", o["g"], C, AM_SCALE, o["a"], hw, o["w3"], C, y, M, C, C, o["b3"], o["x"], o["beta"],
             o["lnw2"], o["lnb2"], n2, st2, EPS, dt)
    else:
        call("gemm_bf16", o["g"], C, AM_SCALE, o["a"], hw, dt, o["w3"], C, y, C, CM_PLAIN, dt, M, C, C, 0, 0, 0,
             o["b3"], o["x"], o["beta"], None)
        call("ln_fwd_nhwc", y, o["lnw2"], o["lnb2"], n2, st2, M, C, EPS, dt)
    call("gemm_bf16", n2, C, AM_PLAIN, None, 1, dt, o["w4"], C, t4, 2 * C, CM_SG, dt, M, 2 * C, C, 0, 0, 0, o["b4"], None,
         None, g2)
    if nxt and C in (128, 256):
        call("gemm_res_ln", g2, C, AM_PLAIN, None, 1, o["w5"], C, out, M, C, C, o["b5"], y, o["gamma"], o["lnw1"],
             o["lnb1"], nn1, nst1, EPS, dt)
    else:
        call("gemm_bf16", g2, C, AM_PLAIN, None, 1, dt, o["w5"], C, out, C, CM_PLAIN, dt, M, C, C, 0, 0, 0, o["b5"], y,
             o["gamma"], None)
        if nxt:
            call("ln_fwd_nhwc", out, o["lnw1"], o["lnb1"], nn1, nst1, M, C, EPS, dt)
    return dict(y=y, n2=n2, st2=st2, t4=t4, g2=g2, out=out, nn1=nn1, nst1=nst1)


CASES = [(128, 2, 4096, True), (128, 1, 1024, False), (256, 2, 1024, True), (256, 3, 256, True), (256, 1, 4096, False),
         (512, 16, 256, False), (512, 2, 256, True), (512, 1, 1024, True)]


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("C,B,hw,nxt", CASES)
def test_ffn_rows_bitwise_equals_the_launches(dev, dt, C, B, hw, nxt):
    from lowlight_image_enhancement_amd._lib import call, query
    M = B * hw
    assert query("ffn_rows_supported", M, C, hw, dt) == 1
    o = _operands(dev, dt, B, hw, C, C + B + hw + dt)
    ref = _reference(dev, dt, M, C, hw, o, nxt)
    Ht = DT[dt]
    # outputs pre-filled with NaN: every element must be written
    nan = lambda *s, dtype=Ht: torch.full(s, float("nan"), device=dev, dtype=dtype)  # noqa: E731
    got = dict(y=nan(M, C), n2=nan(M, C), st2=nan(M, 2, dtype=torch.float32), t4=nan(M, 2 * C), g2=nan(M, C),
               out=nan(M, C), nn1=nan(M, C) if nxt else None,
               nst1=nan(M, 2, dtype=torch.float32) if nxt else None)
    _fused(dev, dt, M, C, hw, o, nxt, got)
    torch.cuda.synchronize()
    for k, v in ref.items():
        if v is None:
            continue
        assert torch.equal(_bits(got[k]), _bits(v)), (k, (got[k].float() - v.float()).abs().max().item())


@pytest.mark.parametrize("dt", [1, 2])
def test_frag16_layout(dev, dt):
    """nbp_frag16: fragment-ordered copies of 16-bit matrices at their flat offsets, bitwise the torch permutation (the
    rest of the buffer untouched)."""
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(3)
    shapes = [(256, 128), (512, 256), (1024, 512), (512, 512), (256, 512)]
    offs, o = [], 8
    for n, k in shapes:
        offs.append(o)
        o += n * k + 8
    src = torch.randn(o, device=dev, generator=gen).to(DT[dt])
    desc = torch.tensor([[of, n, k] for of, (n, k) in zip(offs, shapes)], dtype=torch.int64, device=dev)
    out = torch.full((o,), 7.0, device=dev, dtype=DT[dt])
    call("frag16", src, desc, len(shapes), out)
    torch.cuda.synchronize()
    for of, (n, k) in zip(offs, shapes):
        assert torch.equal(_bits(out[of:of + n * k]), _bits(to_frag(src[of:of + n * k].view(n, k))))
        assert (out[of - 8:of].float() == 7.0).all()


def test_ffn_rows_refusals(dev):
    """Shapes not served: C outside {128, 256, 512}, the fp32 mode, images whose row count is not a multiple of 32 (the
    executor keeps the launches there); a call with such a shape fails loudly."""
    from lowlight_image_enhancement_amd._lib import NBPError, call, query
    assert query("ffn_rows_supported", 4096, 512, 256, 2) == 1
    assert query("ffn_rows_supported", 4096, 64, 256, 2) == 0
    assert query("ffn_rows_supported", 48 * 5, 256, 48, 2) == 0
    assert query("ffn_rows_supported", 4096, 256, 256, 0) == 0
    z = torch.zeros(64, device=dev)
    with pytest.raises(NBPError, match="unsupported shape"):
        call("ffn_rows_fwd", z, z, 48, z, z, z, z, z, z, z, z, z, z, z, None, None, z, z, z, z, z, z, None, None, 48,
             256, EPS, 2)


def _bwd_reference(dev, dt, M, C, hw, o):
    """the launches the executor issued before (nafnet.py _ffn_bwd_launches): conv5 dgrad CM_SGBWD, conv4 dgrad + norm2
    backward (nbp_dgrad_ln_bwd at C 128 / 256; nbp_gemm_bf16 + nbp_ln_bwd_nhwc at C 512), conv3 dgrad CM_CHANDOT"""
    from lowlight_image_enhancement_amd._lib import call, query
    Ht = DT[dt]
    E = lambda n: torch.empty(M, n, device=dev, dtype=Ht)  # noqa: E731
    dt4, dh = E(2 * C), E(C)
    call("gemm_bf16", o["dout"], C, AM_PLAIN, None, 1, dt, o["w5t"], C, dt4, 2 * C, CM_SGBWD, dt, M, C, C, 0, 0, 0, None,
         o["t4"], None, None)
    dy, dlnw, dlnb = _dgrad_ln_reference(dev, dt, M, C, dt4, o["w4t"], o["y"], o["st2"], o["lnw2"], o["dout"])
    B = M // hw
    da = torch.empty(B * (hw // 64) * C, device=dev)
    call("gemm_bf16", dy, C, AM_PLAIN, None, hw, dt, o["w3t"], C, dh, C, CM_CHANDOT, dt, M, C, C, 0, 0, 0, None, o["g"],
         None, da)
    return dict(dt4=dt4, dy=dy, dh=dh, dlnw=dlnw, dlnb=dlnb, da=da.view(B, hw // 64, C).sum(1))


def _dgrad_ln_reference(dev, dt, M, C, d, wt, x, st, lnw, dres):
    """the (K = 2C) input gradient + LayerNorm2d backward + residual as the executor launches it (nafnet.py
    _conv1_bwd / _ffn_bwd_launches): nbp_dgrad_ln_bwd at C 128 / 256, nbp_gemm_bf16 + nbp_ln_bwd_nhwc at C 512.
    Returns (dx, d weight, d bias)."""
    from lowlight_image_enhancement_amd._lib import call, query
    out = torch.empty(M, C, device=dev, dtype=DT[dt])
    dlnw, dlnb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    if C in (128, 256):
        n_ws = query("dgrad_ln_workspace_floats", M, C)
        ws = torch.empty(n_ws, device=dev)
        call("dgrad_ln_bwd", d, 2 * C, wt, 2 * C, M, C, 2 * C, x, st, lnw, dres, out, dlnw, dlnb, ws, n_ws, dt)
    else:
        dn = torch.empty(M, C, device=dev, dtype=DT[dt])
        call("gemm_bf16", d, 2 * C, AM_PLAIN, None, 1, dt, wt, 2 * C, dn, C, CM_PLAIN, dt, M, C, 2 * C, 0, 0, 0,
             None, None, None, None)
        lg = query("ln_nhwc_grid", M, C, dt)
        sw, sb = torch.empty(lg * C, device=dev), torch.empty(lg * C, device=dev)
        call("ln_bwd_nhwc", dn, x, st, lnw, dres, out, sw, sb, M, C, dt)
        call("reduce_slab", sw, lg, C, dlnw)
        call("reduce_slab", sb, lg, C, dlnb)
    return out, dlnw, dlnb


def _ln_input(R, M, C, Ht):
    x = (R(M, C) * 1.5 + 0.2).to(Ht)
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    den = ((xd - mu) ** 2).mean(1, keepdim=True).add(1e-6).sqrt()
    return x, torch.cat([mu, den], 1).float().contiguous()


CM_SGBWD, CM_CHANDOT = 5, 8


@pytest.mark.parametrize("pre", [False, True])
@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("C,B,hw", [(128, 2, 4096), (128, 1, 1024), (256, 2, 1024), (256, 3, 256), (512, 16, 256),
                                    (512, 1, 1024)])
def test_ffn_rows_bwd_bitwise_equals_the_launches(dev, dt, C, B, hw, pre):
    """nbp_ffn_rows_bwd: dt4, dy, dh bitwise the launches it replaces; the norm2 weight / bias gradients and the SCA
    channel dot (its per-32-row partials summed per image) within fp32 summation order of theirs.  pre: dout is made
    in the launch as the following block's dx (its conv1 input gradient + norm1 backward + residual), bitwise
    _dgrad_ln_reference, norm1's weight / bias gradients within fp32 summation order."""
    from lowlight_image_enhancement_amd._lib import call
    Ht = DT[dt]
    M = B * hw
    gen = torch.Generator(device=dev).manual_seed(C + B + hw + 7 * dt)
    R = lambda *s: torch.randn(*s, device=dev, generator=gen)  # noqa: E731
    y, st2 = _ln_input(R, M, C, Ht)
    o = dict(dout=R(M, C).to(Ht), t4=R(M, 2 * C).to(Ht), y=y, st2=st2, lnw2=1 + 0.1 * R(C), g=R(M, C).to(Ht),
             w5t=(R(C, C) / C ** 0.5).to(Ht), w4t=(R(C, 2 * C) / C ** 0.5).to(Ht), w3t=(R(C, C) / C ** 0.5).to(Ht))
    nan = lambda *s: torch.full(s, float("nan"), device=dev, dtype=Ht)  # noqa: E731
    nb = M // 32
    pre_args, ref1 = (None,) * 9, None
    if pre:
        x1, st1 = _ln_input(R, M, C, Ht)
        q = dict(dt1=R(M, 2 * C).to(Ht), w1t=(R(C, 2 * C) / C ** 0.5).to(Ht), x1=x1, st1=st1, lnw1=1 + 0.1 * R(C),
                 dres1=R(M, C).to(Ht))
        ref1 = _dgrad_ln_reference(dev, dt, M, C, q["dt1"], q["w1t"], x1, st1, q["lnw1"], q["dres1"])
        o["dout"] = ref1[0]
        dx1 = nan(M, C)
        sw1, sb1 = (torch.full((nb * C,), float("nan"), device=dev) for _ in range(2))
        pre_args = (q["dt1"], to_frag(q["w1t"]), x1, st1, q["lnw1"], q["dres1"], dx1, sw1, sb1)
    ref = _bwd_reference(dev, dt, M, C, hw, o)
    got = dict(dt4=nan(M, 2 * C), dy=nan(M, C), dh=nan(M, C))
    sw, sb, da = (torch.full((nb * C,), float("nan"), device=dev) for _ in range(3))
    call("ffn_rows_bwd", None if pre else o["dout"], o["t4"], o["y"], o["st2"], o["lnw2"], o["g"], to_frag(o["w5t"]),
         to_frag(o["w4t"]), to_frag(o["w3t"]), got["dt4"], got["dy"], got["dh"], sw, sb, da, *pre_args, M, C, hw, dt)
    torch.cuda.synchronize()
    if pre:
        assert torch.equal(_bits(dx1), _bits(ref1[0])), (dx1.float() - ref1[0].float()).abs().max().item()
        for v, r in ((sw1.view(nb, C).sum(0), ref1[1]), (sb1.view(nb, C).sum(0), ref1[2])):
            assert (v - r).abs().max().item() <= 2e-5 * r.abs().max().item() + 1e-6
    for k in ("dt4", "dy", "dh"):
        assert torch.equal(_bits(got[k]), _bits(ref[k])), (k, (got[k].float() - ref[k].float()).abs().max().item())
    for k, v in (("dlnw", sw.view(nb, C).sum(0)), ("dlnb", sb.view(nb, C).sum(0)),
                 ("da", da.view(B, hw // 32, C).sum(1))):
        r = ref[k]
        assert (v - r).abs().max().item() <= 2e-5 * r.abs().max().item() + 1e-6, k


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_ffn_rows_network(dev, precision):
    """Width 32, four downs at 128^2: levels 2 (32^2, C 128), 3 (16^2, C 256) and the middle (8^2 = 64 rows, C 512) take
    the fused launches (forward and backward): the output bitwise that of the unfused network; every parameter gradient
    within the 16-bit rounding that the partial sums' fp32 order can move (the SCA gradient enters the depthwise
    backward's 16-bit dt2)."""
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    torch.manual_seed(9)
    net = create_newbp_net(in_channels=3, width=32, enc_blk_nums=[1, 1, 2, 2], middle_blk_num=2,
                           dec_blk_nums=[1, 1, 1, 1]).to(dev)
    net.precision = precision
    with torch.no_grad():
        net.flat.add_(torch.randn_like(net.flat) * 0.02)
    x = torch.rand(2, 3, 128, 128, device=dev)
    res = []
    for fuse in (True, False):
        net.fuse_ffn_rows = fuse
        net.flat.grad = None
        out = net(x)
        out.square().mean().backward()
        res.append((out.detach().clone(), net.flat.grad.clone()))
    net.fuse_ffn_rows = True
    (o1, g1), (o0, g0) = res
    assert torch.equal(o1, o0)
    assert (g1 - g0).norm().item() <= 2e-3 * g0.norm().item()
