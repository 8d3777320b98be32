"""The level-0 / 1 tile forward (nbp_c1dw_fwd_tile, NAFNet_arch.py:59-68) against float64 stage by stage, from the
kernel's own 16-bit intermediates (its t1 / t2-keeping form): t1 = conv1(n1) + b1, t2 = depthwise 3x3 (zero padding
1) of t1 + bias, g = t2[:C] t2[C:] (the product of the fp32 depthwise outputs, before their rounding) -- each within
one 16-bit ulp (+ the fp32
accumulation allowance of test_gpu_ffn_rows_f64._within_ulp).  Independent of the two-launch path the tile kernels
are pinned to bitwise in test_gpu_c1dw_tile.py."""
import pytest
import torch
import torch.nn.functional as Fn

from test_gpu_c1dw_tile import DT, SHAPES, _operands
from test_gpu_ffn_rows_f64 import _within_ulp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("B,H,W,C", SHAPES)
def test_fwd_tile_against_float64(dev, dt, B, H, W, C):
    from lowlight_image_enhancement_amd._lib import call, query
    Ht, M = DT[dt], B * H * W
    n1, w1, b1, wdw, bdw = _operands(dev, dt, B, H, W, C, 7 + B + H + W + C + dt)
    rows = query("c1dw_tile_rows", H, W, C)
    t1, t2, g = (torch.empty(M, n, device=dev, dtype=Ht) for n in (2 * C, 2 * C, C))
    pool = torch.empty(B * rows * C, device=dev)
    call("c1dw_fwd_tile", n1, w1, b1, wdw, bdw, t1, t2, g, pool, B, H, W, C, dt)
    torch.cuda.synchronize()
    D = lambda t: t.double()  # noqa: E731
    _within_ulp(t1, D(n1) @ D(w1).T + D(b1), dt, "t1")
    t1d = D(t1).view(B, H, W, 2 * C).permute(0, 3, 1, 2)
    t2d = Fn.conv2d(t1d, D(wdw).view(2 * C, 1, 3, 3), D(bdw), padding=1, groups=2 * C)
    t2r = t2d.permute(0, 2, 3, 1).reshape(M, 2 * C)
    _within_ulp(t2, t2r, dt, "t2")
    _within_ulp(g, t2r[:, :C] * t2r[:, C:], dt, "g")
