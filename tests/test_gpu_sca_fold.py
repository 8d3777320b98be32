"""nbp_sca_dw_bwd: the SCA backward (NAFNet_arch.py:39-41, 67 -- ds = W_sca^T da, dW_sca = da^T mean, db_sca = sum_b
da) folded into the fused depthwise backward, against the two launches it replaces (nbp_sca_bwd_fused +
nbp_sca_sg_dw_bwd) at the stored-tape levels' shapes.

Exact case: the channel-dot partials, W_sca and the means are small dyadic numbers, so every fp32 sum of the SCA
backward is exact in any order: ds, dW_sca, db_sca and hence dt1 and the depthwise gradients must be bitwise those of
the two launches.  Random case: the fold's own summation orders move ds in the last fp32 bits; dW_sca / db_sca within
fp32 summation order, dt1 within one 16-bit rounding of the SimpleGate product (dt2) per tap."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DT = {1: torch.bfloat16, 2: torch.float16}


def _bits(t):
    return t.view(torch.int16) if t.dtype in (torch.float16, torch.bfloat16) else t.view(torch.int32)


def _case(dev, dt, B, H, W, C, exact, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    I = lambda lo, hi, *s: torch.randint(lo, hi, s, device=dev, generator=g).float()  # noqa: E731
    Ht = DT[dt]
    M, HW = B * H * W, H * W
    chunks = HW // 32
    o = dict(dh=R(M, C).to(Ht), a=torch.rand(B, C, device=dev, generator=g) + 0.5, t2=R(M, 2 * C).to(Ht),
             t1=R(M, 2 * C).to(Ht), wdw=R(2 * C, 9) * 0.3)
    if exact:
        o["da"] = I(-8, 9, B * chunks * C) * 2.0 ** -6
        o["wsca"] = I(-8, 9, C, C) * 2.0 ** -8
        o["mean"] = I(-8, 9, B, C) * 2.0 ** -6
    else:
        o["da"] = R(B * chunks * C)
        o["wsca"] = R(C, C) / C ** 0.5
        o["mean"] = R(B, C)
    return o, chunks


def _run(dev, dt, B, H, W, C, o, chunks, fold):
    from lowlight_image_enhancement_amd._lib import call, query
    M = B * H * W
    dt1 = torch.full((M, 2 * C), float("nan"), device=dev, dtype=DT[dt])
    dwdw, dbdw = torch.zeros(2 * C * 9, device=dev), torch.zeros(2 * C, device=dev)
    dws, dbs = torch.full((C * C,), float("nan"), device=dev), torch.full((C,), float("nan"), device=dev)
    ws = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
    if fold:
        call("sca_dw_bwd", o["dh"], o["a"], o["da"], chunks, o["wsca"], o["mean"], dws, dbs, o["t2"], o["t1"], o["wdw"],
             dt1, dwdw, dbdw, ws, B, H, W, C, dt)
    else:
        ds = torch.empty(B, C, device=dev)
        call("sca_bwd_fused", o["da"], chunks, o["wsca"], o["mean"], ds, dws, dbs, B, C)
        call("sca_sg_dw_bwd", o["dh"], o["a"], ds, o["t2"], o["t1"], o["wdw"], dt1, dwdw, dbdw, ws, B, H, W, C, dt)
    torch.cuda.synchronize()
    return dict(dt1=dt1, dwdw=dwdw, dbdw=dbdw, dws=dws, dbs=dbs)


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", [(16, 16, 16, 512), (16, 32, 32, 256), (4, 64, 64, 128), (3, 16, 48, 256)])
def test_sca_fold_exact_bitwise(dev, dt, B, H, W, C):
    o, chunks = _case(dev, dt, B, H, W, C, True, 3 + C + B)
    got, ref = _run(dev, dt, B, H, W, C, o, chunks, True), _run(dev, dt, B, H, W, C, o, chunks, False)
    for k in ("dt1", "dws", "dbs"):
        assert torch.equal(_bits(got[k]), _bits(ref[k])), k
    for k in ("dwdw", "dbdw"):  # per-tile partials, the same kernel body: bitwise too
        assert torch.equal(_bits(got[k]), _bits(ref[k])), k


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", [(16, 16, 16, 512), (16, 32, 32, 256)])
def test_sca_fold_random_within_rounding(dev, dt, B, H, W, C):
    o, chunks = _case(dev, dt, B, H, W, C, False, 11 + C)
    got, ref = _run(dev, dt, B, H, W, C, o, chunks, True), _run(dev, dt, B, H, W, C, o, chunks, False)
    for k in ("dws", "dbs"):
        r = ref[k]
        assert (got[k] - r).abs().max().item() <= 1e-5 * r.abs().max().item(), k
    # ds moves by fp32 ulps: a dt2 = (H)(dg * t2) can round the other way, 1 ulp of the 16-bit type, weighted by the
    # taps into dt1 (9 taps, |w| <~ 1)
    eps = torch.finfo(DT[dt]).eps
    d = (got["dt1"].float() - ref["dt1"].float()).abs()
    assert d.max().item() <= 9 * 2 * eps * ref["dt1"].float().abs().max().item() + 1e-6
    assert (d > 0).float().mean().item() < 0.05
    for k in ("dwdw", "dbdw"):
        r = ref[k]
        assert (got[k] - r).abs().max().item() <= 1e-2 * r.abs().max().item(), k


def _run_tile(dev, dt, B, H, W, C, o, chunks, fold):
    from lowlight_image_enhancement_amd._lib import call, query
    M = B * H * W
    dt1 = torch.full((M, 2 * C), float("nan"), device=dev, dtype=DT[dt])
    dwdw, dbdw = torch.zeros(2 * C * 9, device=dev), torch.zeros(2 * C, device=dev)
    dws, dbs = torch.full((C * C,), float("nan"), device=dev), torch.full((C,), float("nan"), device=dev)
    ws = torch.empty(query("c1dw_bwd_workspace_floats", B, H, W, C), device=dev)
    tail = (o["n1"], o["w1"], o["b1"], o["wdw"], o["bdw"], dt1, dwdw, dbdw, ws, B, H, W, C, dt)
    if fold:
        call("sca_c1dw_bwd_tile", o["dh"], o["a"], o["da"], chunks, o["wsca"], o["mean"], dws, dbs, *tail)
    else:
        ds = torch.empty(B, C, device=dev)
        call("sca_bwd_fused", o["da"], chunks, o["wsca"], o["mean"], ds, dws, dbs, B, C)
        call("c1dw_bwd_tile", o["dh"], o["a"], ds, *tail)
    torch.cuda.synchronize()
    return dict(dt1=dt1, dwdw=dwdw, dbdw=dbdw, dws=dws, dbs=dbs)


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", [(2, 64, 64, 32), (3, 40, 72, 32), (2, 64, 64, 64), (16, 32, 32, 64)])
def test_sca_fold_tile_exact_bitwise(dev, dt, B, H, W, C):
    """the same fold in the level-0 / 1 tile backward (nbp_sca_c1dw_bwd_tile vs nbp_sca_bwd_fused +
    nbp_c1dw_bwd_tile): exact dyadic SCA inputs, everything bitwise"""
    o, chunks = _case(dev, dt, B, H, W, C, True, 5 + C + H)
    g = torch.Generator(device=dev).manual_seed(77 + C)
    R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    o.update(n1=R(B * H * W, C).to(DT[dt]), w1=(R(2 * C, C) / C ** 0.5).to(DT[dt]), b1=R(2 * C) * 0.1,
             bdw=R(2 * C) * 0.1)
    got, ref = _run_tile(dev, dt, B, H, W, C, o, chunks, True), _run_tile(dev, dt, B, H, W, C, o, chunks, False)
    for k in ("dt1", "dws", "dbs", "dwdw", "dbdw"):
        assert torch.equal(_bits(got[k]), _bits(ref[k])), k
