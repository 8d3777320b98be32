"""The level-0 NAFBlock FFN half in one pass (nbp_gemm_ffn; reference NAFNet_arch.py:74-80):
conv4 -> SimpleGate -> conv5 + layer-scale residual (+ the next block's LayerNorm2d) with the gate map g2 kept in
registers.  It must be bitwise the two-launch form it replaces (nbp_gemm_bf16 CM_SG, then nbp_gemm_res_ln or the
residual GEMM) on ragged row counts, in both 16-bit types, and close to float64 torch on the same rounded operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CM_PLAIN, CM_SG = 0, 4


def _operands(dev, M, dt, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    H = torch.bfloat16 if dt == 1 else torch.float16
    C = 32
    n2 = torch.randn(M, C, device=dev, generator=g).to(H)
    y = torch.randn(M, C, device=dev, generator=g).to(H)
    W4 = (torch.randn(2 * C, C, device=dev, generator=g) * 0.3).to(H)  # rows already SimpleGate-interleaved
    b4 = torch.randn(2 * C, device=dev, generator=g) * 0.1
    W5 = (torch.randn(C, C, device=dev, generator=g) * 0.3).to(H)
    b5 = torch.randn(C, device=dev, generator=g) * 0.1
    gamma = torch.randn(C, device=dev, generator=g) * 0.5
    lnw = torch.rand(C, device=dev, generator=g) + 0.5
    lnb = torch.randn(C, device=dev, generator=g) * 0.1
    return H, C, n2, y, W4, b4, W5, b5, gamma, lnw, lnb


@pytest.mark.parametrize("dt", [1, 2])
@pytest.mark.parametrize("M", [32, 1000, 4096, 65536 + 17])
@pytest.mark.parametrize("with_ln", [True, False])
def test_ffn_bitwise_equals_two_launches(dev, dt, M, with_ln):
    from lowlight_image_enhancement_amd._lib import call
    H, C, n2, y, W4, b4, W5, b5, gamma, lnw, lnb = _operands(dev, M, dt, M + 7 * dt)
    eps = 1e-6
    # two launches: conv4 with the SimpleGate epilogue (t4 dropped), then conv5 (+ residual, + LN)
    g2 = torch.empty(M, C, device=dev, dtype=H)
    call("gemm_bf16", n2, C, 0, None, 1, dt, W4, C, None, 2 * C, CM_SG, dt, M, 2 * C, C, 0, 0, 0, b4, None, None, g2)
    ref_out = torch.empty(M, C, device=dev, dtype=H)
    ref_n, ref_st = torch.empty(M, C, device=dev, dtype=H), torch.empty(M, 2, device=dev)
    if with_ln:
        call("gemm_res_ln", g2, C, 0, None, 1, W5, C, ref_out, M, C, C, b5, y, gamma, lnw, lnb, ref_n, ref_st, eps, dt)
    else:
        call("gemm_bf16", g2, C, 0, None, 1, dt, W5, C, ref_out, C, CM_PLAIN, dt, M, C, C, 0, 0, 0, b5, y, gamma, None)
    out = torch.empty(M, C, device=dev, dtype=H)
    nn, st = torch.empty(M, C, device=dev, dtype=H), torch.empty(M, 2, device=dev)
    call("gemm_ffn", n2, W4, b4, W5, b5, y, gamma, lnw if with_ln else None, lnb if with_ln else None, out,
         nn if with_ln else None, st if with_ln else None, M, C, eps, dt)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref_out.view(torch.int16))
    if with_ln:
        assert torch.equal(nn.view(torch.int16), ref_n.view(torch.int16))
        assert torch.equal(st, ref_st)
    # and against float64 torch on the same rounded operands (the 16-bit roundings of t4 / g2 / out aside)
    t = n2.double() @ W4.double().t() + b4.double()
    gate = (t[:, 0::2] * t[:, 1::2]).to(H).double()
    ref64 = y.double() + gamma.double() * (gate @ W5.double().t() + b5.double())
    tol = 4e-2 if dt == 1 else 5e-3
    assert ((out.double() - ref64).abs() <= tol * (1 + ref64.abs())).all()


def test_ffn_rejects_other_widths(dev):
    from lowlight_image_enhancement_amd._lib import NBPError, call
    H, C, n2, y, W4, b4, W5, b5, gamma, lnw, lnb = _operands(dev, 64, 1, 3)
    out = torch.empty(64, C, device=dev, dtype=H)
    with pytest.raises(NBPError, match="C = 32"):
        call("gemm_ffn", n2, W4, b4, W5, b5, y, gamma, None, None, out, None, None, 64, 64, 1e-6, 1)
