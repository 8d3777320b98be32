"""Image-boundary conv weight gradients (nbp_intro_bwd / nbp_ending_bwd, NAFNet_arch.py:88-91,134-136) against
float64 torch on the same stored operands, at cfg2's level 0, padded grids (check_image_size), cfg3's 512-wide rows,
w64 and 1-channel images, in every storage mode."""
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu

# (B, Cimg, H0, W0, Hp, Wp, Cf): cfg2 level 0, a padded grid (check_image_size), cfg3's 512-wide rows, w64, 1 channel
SHAPES = [(2, 3, 256, 256, 256, 256, 32), (2, 3, 61, 45, 64, 48, 16), (1, 3, 512, 512, 512, 512, 32),
          (2, 3, 64, 64, 64, 64, 64), (2, 1, 40, 40, 40, 40, 24), (3, 3, 33, 200, 40, 200, 40)]


def _run(dev, B, CI, H0, W0, Hp, Wp, Cf, dtype):
    from lowlight_image_enhancement_amd._lib import call, query
    td = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[dtype]
    gen = torch.Generator(device=dev).manual_seed(B + H0 * W0 + Cf + dtype)
    img = torch.rand(B, CI, H0, W0, device=dev, generator=gen)
    dout = torch.randn(B, Hp, Wp, Cf, device=dev, generator=gen).to(td)
    w = torch.randn(Cf, CI, 3, 3, device=dev, generator=gen)
    dy = torch.randn(B, CI, H0, W0, device=dev, generator=gen)
    feat = torch.randn(B, Hp, Wp, Cf, device=dev, generator=gen).to(td)
    we = torch.randn(CI, Cf, 3, 3, device=dev, generator=gen)
    dw_i, db_i = torch.empty_like(w), torch.empty(Cf, device=dev)
    dw_e, db_e = torch.empty_like(we), torch.empty(CI, device=dev)
    dfeat = torch.empty(B, Hp, Wp, Cf, device=dev, dtype=td)
    ws = torch.empty(max(query("intro_bwd_workspace_floats", B, CI, Hp, Wp, Cf),
                         query("ending_bwd_workspace_floats", B, CI, H0, W0, Cf)), device=dev)
    call("intro_bwd", img, dout, w, dw_i, db_i, None, ws, B, CI, H0, W0, Hp, Wp, Cf, dtype)
    call("ending_bwd", dy, feat, we, dfeat, dw_e, db_e, ws, B, CI, H0, W0, Hp, Wp, Cf, dtype)
    torch.cuda.synchronize()
    # ending input gradient: dfeat = conv_transpose(dy zero-padded to the grid) on the stored weights
    dyp = Fn.pad(dy.double(), (0, Wp - W0, 0, Hp - H0))
    ref_dfeat = Fn.conv_transpose2d(dyp, we.double(), padding=1).permute(0, 2, 3, 1)
    err = (dfeat.double() - ref_dfeat).abs().max().item()
    tol = 1e-5 if dtype == 0 else (2.0 ** -8 if dtype == 1 else 2.0 ** -11) * 2
    assert err <= tol * ref_dfeat.abs().max().item() + 1e-6, ("dfeat", err)
    return (img, dout, dy, feat), (dw_i, db_i, dw_e, db_e)


@pytest.mark.parametrize("dtype", [0, 1, 2], ids=["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("shape", SHAPES, ids=["x".join(map(str, s)) for s in SHAPES])
def test_boundary_conv_gradients_against_float64(dev, shape, dtype):
    B, CI, H0, W0, Hp, Wp, Cf = shape
    if dtype and Cf % 8:
        pytest.skip("16-bit widths are multiples of 8")
    (img, dout, dy, feat), new = _run(dev, B, CI, H0, W0, Hp, Wp, Cf, dtype)
    # float64 reference on the stored operands: intro y = conv(img zero-padded to Hp x Wp), ending y = conv(feat)
    # cropped to H0 x W0 (dy zero off the crop)
    imgp = Fn.pad(img.double(), (0, Wp - W0, 0, Hp - H0))
    g = dout.double().permute(0, 3, 1, 2)
    ref_dw_i = torch.nn.grad.conv2d_weight(imgp, (Cf, CI, 3, 3), g, padding=1)
    ref_db_i = g.sum((0, 2, 3))
    dyp = Fn.pad(dy.double(), (0, Wp - W0, 0, Hp - H0))
    ref_dw_e = torch.nn.grad.conv2d_weight(feat.double().permute(0, 3, 1, 2), (CI, Cf, 3, 3), dyp, padding=1)
    ref_db_e = dy.double().sum((0, 2, 3))
    for name, a, r in zip(("dw_intro", "db_intro", "dw_ending", "db_ending"), new, (ref_dw_i, ref_db_i, ref_dw_e,
                                                                                     ref_db_e)):
        err = (a.double() - r).abs().max().item()
        assert err <= 1e-5 * r.abs().max().item() + 1e-6, (name, err)


@pytest.mark.parametrize("dtype", [0, 1, 2], ids=["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("shape", SHAPES, ids=["x".join(map(str, s)) for s in SHAPES])
def test_boundary_conv_lds_staging_bitwise(dev, shape, dtype, monkeypatch):
    """The LDS-staged weight-gradient kernel runs each wave's pixel-pair sequence of the gather kernel: every slab, so
    dW / db, is bitwise the gather kernel's (NBP_BCONV_GATHER=1, read per launch)."""
    B, CI, H0, W0, Hp, Wp, Cf = shape
    if dtype and Cf % 8:
        pytest.skip("16-bit widths are multiples of 8")
    _, staged = _run(dev, B, CI, H0, W0, Hp, Wp, Cf, dtype)
    monkeypatch.setenv("NBP_BCONV_GATHER", "1")
    _, gather = _run(dev, B, CI, H0, W0, Hp, Wp, Cf, dtype)
    for name, a, r in zip(("dw_intro", "db_intro", "dw_ending", "db_ending"), staged, gather):
        assert torch.equal(a.view(torch.int32), r.view(torch.int32)), name
