"""The per-step 16-bit weight copies (nbp_weights_bf16): the straight copy is the flat fp32 buffer rounded, each listed
matrix's transposed copy is (diag(s) W)^T rounded (s the conv3 / conv5 layer scale when one is listed), bitwise equal
to torch on the same values, for every GEMM weight of the cfg2 network and for ragged shapes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [1, 2])
def test_weight_copies_cfg2_bitwise(dev, dt):
    from lowlight_image_enhancement_amd._lib import call
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    H = {1: torch.bfloat16, 2: torch.float16}[dt]
    net = create_newbp_net(in_channels=3, width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12,
                           dec_blk_nums=[2, 2, 2, 2]).to(dev)
    torch.manual_seed(0)
    flat = torch.randn(net.numel, device=dev)
    desc = net._tdesc_cpu.to(dev)
    wb = torch.full((net.numel,), float("nan"), dtype=H, device=dev)
    wt = torch.full((net.numel,), float("nan"), dtype=H, device=dev)
    call("weights_bf16", flat, net.numel, wb, desc, desc.shape[0], wt, dt)
    torch.cuda.synchronize()
    assert torch.equal(wb.view(torch.int16), flat.to(H).view(torch.int16))
    for off, R, C, soff in net._tdesc_cpu.tolist():
        W = flat[off:off + R * C].view(R, C)
        if soff >= 0:
            W = W * flat[soff:soff + R].view(R, 1)
        assert torch.equal(wt[off:off + R * C].view(torch.int16), W.t().contiguous().to(H).view(-1).view(torch.int16))


@pytest.mark.parametrize("R,C,scaled", [(8, 12, False), (72, 100, True), (130, 66, False), (5, 7, True)])
def test_weight_copies_ragged(dev, R, C, scaled):
    from lowlight_image_enhancement_amd._lib import call
    n = 4 + R * C + R + 3  # a leading pad, the matrix, its row scale, an odd tail
    flat = torch.randn(n, device=dev)
    desc = torch.tensor([[4, R, C, 4 + R * C if scaled else -1]], dtype=torch.int64, device=dev)
    wb = torch.zeros(n, dtype=torch.float16, device=dev)
    wt = torch.zeros(n, dtype=torch.float16, device=dev)
    call("weights_bf16", flat, n, wb, desc, 1, wt, 2)
    torch.cuda.synchronize()
    assert torch.equal(wb, flat.half())
    W = flat[4:4 + R * C].view(R, C)
    if scaled:
        W = W * flat[4 + R * C:4 + R * C + R].view(R, 1)
    assert torch.equal(wt[4:4 + R * C], W.t().contiguous().half().view(-1))
