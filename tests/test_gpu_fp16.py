"""fp16 mode (dtype 2: fp16 activation storage and v_mfma_f32_32x32x16_f16 operands, fp32 accumulation) -- the
reference's autocast dtype (image_restoration_model.py:255, GradScaler :104-106,308-320).

Kernel level: every 16-bit entry point on fp16 operands against float64 math on the same fp16-rounded operands.
Network level: the cfg2 / w64 models against the reference's fp32 outputs (the reference's own forward under
torch.autocast(float16) reaches 48.0 dB at cfg2, measured on CPU in the build container), and the VGG19 input gradient
at full depth under the trainer's loss scale against bf16's.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
T = torch.from_numpy
H16 = torch.float16


def _rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm()).item()


@pytest.mark.parametrize("M,N,K", [(4096, 1024, 512), (1000, 64, 32), (300, 40, 72), (333, 48, 24), (70000, 256, 128)])
def test_gemm_fp16_tiled_and_skinny(dev, M, N, K):
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev, generator=gen).to(H16)
    W = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(H16)
    bias = torch.randn(N, device=dev, generator=gen)
    out = torch.empty(M, N, device=dev, dtype=H16)
    call("gemm_bf16", A, K, 0, None, 1, 2, W, K, out, N, 0, 2, M, N, K, 0, 0, 0, bias, None, None, None)
    ref = A.double() @ W.double().t() + bias.double()
    assert (out.double() - ref).abs().max().item() <= 2e-3 * ref.abs().max().item() + 2e-3
    # fp32 A / fp32 C with fp16 weights is not a mode (fp32 in and out selects bf16 weights): mixed dtypes refused
    with pytest.raises(Exception):
        call("gemm_bf16", A.to(torch.bfloat16), K, 0, None, 1, 1, W, K, out, N, 0, 2, M, N, K, 0, 0, 0, None, None,
             None, None)


@pytest.mark.parametrize("M,C", [(1000, 32), (4096, 64), (300, 24)])
def test_gemm_fp16_simplegate_epilogues(dev, M, C):
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(M + C)
    K = C
    A = torch.randn(M, K, device=dev, generator=gen).to(H16)
    W = (torch.randn(2 * C, K, device=dev, generator=gen) * 0.2).to(H16)
    b = torch.randn(2 * C, device=dev, generator=gen)
    t = torch.empty(M, 2 * C, device=dev, dtype=H16)
    g = torch.empty(M, C, device=dev, dtype=H16)
    call("gemm_bf16", A, K, 0, None, 1, 2, W, K, t, 2 * C, 4, 2, M, 2 * C, K, 0, 0, 0, b, None, None, g)
    tr = A.double() @ W.double().t() + b.double()
    assert (t.double() - tr).abs().max().item() <= 1e-3 * tr.abs().max().item() + 1e-3
    gr = t.double()[:, 0::2] * t.double()[:, 1::2]
    assert (g.double() - gr).abs().max().item() <= 1e-3 * gr.abs().max().item() + 1e-3


@pytest.mark.parametrize("M,N,K", [(4096, 32, 64), (3000, 64, 128), (4096, 128, 256), (2048, 256, 512),
                                   (4096, 512, 1024)])
def test_dgrad_ln_bwd_fp16(dev, M, N, K):
    """The dgrad + LayerNorm2d-backward fusion on fp16 storage vs float64 (arch_util.py:277-289)."""
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(M + N + K + 2)
    A = torch.randn(M, K, device=dev, generator=gen).to(H16)
    Wt = (torch.randn(N, K, device=dev, generator=gen) / K ** 0.5).to(H16)
    x = (torch.randn(M, N, device=dev, generator=gen) * 2 + 0.5).to(H16)
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    den = ((xd - mu) ** 2).mean(1, keepdim=True).add(1e-6).sqrt()
    stats = torch.cat([mu, den], 1).float().contiguous()
    lnw = torch.rand(N, device=dev, generator=gen) + 0.5
    dres = torch.randn(M, N, device=dev, generator=gen).to(H16)
    dx = torch.empty(M, N, device=dev, dtype=H16)
    dlnw, dlnb = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
    n_ws = query("dgrad_ln_workspace_floats", M, N)
    ws = torch.empty(n_ws, device=dev)
    call("dgrad_ln_bwd", A, K, Wt, K, M, N, K, x, stats, lnw, dres, dx, dlnw, dlnb, ws, n_ws, 2)
    dn = A.double() @ Wt.double().t()
    yh = (xd - mu) / stats[:, 1:2].double()
    g = dn * lnw.double()
    ref = (g - yh * (g * yh).mean(1, keepdim=True) - g.mean(1, keepdim=True)) / stats[:, 1:2].double() + dres.double()
    assert (dx.double() - ref).abs().max().item() <= 2e-3 * ref.abs().max().item() + 2e-3
    assert (dlnw.double() - (dn * yh).sum(0)).abs().max().item() <= 1e-3 * (dn * yh).abs().sum(0).max().item()
    assert (dlnb.double() - dn.sum(0)).abs().max().item() <= 1e-3 * dn.abs().sum(0).max().item()


@pytest.mark.parametrize("M,N,K", [(4096, 64, 128), (70000, 128, 64), (8192, 256, 256)])
def test_wgrad_fp16(dev, M, N, K):
    from lowlight_image_enhancement_amd._lib import call, query
    gen = torch.Generator(device=dev).manual_seed(M + N + K + 3)
    G = torch.randn(M, N, device=dev, generator=gen).to(H16)
    X = torch.randn(M, K, device=dev, generator=gen).to(H16)
    dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    n_ws = query("wgrad_workspace_floats", M, N, K)
    ws = torch.empty(n_ws, device=dev)
    call("wgrad_f32", G, N, 0, X, K, 0, None, 1, M, N, K, 0, 0, 0, 0, dW, db, ws, n_ws, 2)
    ref = G.double().t() @ X.double()
    assert (dW.double() - ref).abs().max().item() <= 1e-4 * M ** 0.5
    assert (db.double() - G.double().sum(0)).abs().max().item() <= 1e-4 * M ** 0.5


def test_conv3x3_fp16(dev):
    import torch.nn.functional as Fn
    from lowlight_image_enhancement_amd._lib import call
    gen = torch.Generator(device=dev).manual_seed(7)
    B, H, W, Cin, Cout = 2, 13, 17, 16, 24
    x = torch.randn(B, H, W, Cin, device=dev, generator=gen).to(H16)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev, generator=gen) / (9 * Cin) ** 0.5)
    b = torch.randn(Cout, device=dev, generator=gen)
    wf = w.permute(0, 2, 3, 1).reshape(Cout, 9, Cin).to(H16).contiguous()
    y = torch.empty(B, H, W, Cout, device=dev, dtype=H16)
    call("conv3x3_bf16", x, B, H, W, Cin, wf, Cout, b, 0, None, y, 1, 2)
    wr = wf.double().view(Cout, 3, 3, Cin).permute(0, 3, 1, 2)
    ref = Fn.relu(Fn.conv2d(x.double().permute(0, 3, 1, 2), wr, b.double(), padding=1)).permute(0, 2, 3, 1)
    assert (y.double() - ref).abs().max().item() <= 2e-3 * ref.abs().max().item() + 1e-3


# ---------------------------------------------------------------------------------------------- network level
CFG2 = dict(width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
CFG4 = dict(width=64, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])


def _net(cfg, seed, dev, precision):
    from param_recipe import recipe_state
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    net = create_newbp_net(in_channels=3, kernel_type="rgb", kernel_spec="B2", **cfg)
    net.load_state_dict(recipe_state([(k, tuple(v.shape)) for k, v in net.state_dict().items()], seed))
    net = net.to(dev)
    net.precision = precision
    return net


def _psnr(a, b):
    mse = ((a.double() - b.double()) ** 2).mean().item()
    return 10 * np.log10(1.0 / mse)


@pytest.mark.parametrize("fixture,cfg", [("nafnet_cfg2.npz", CFG2), ("nafnet_w64.npz", CFG4)])
def test_fp16_mode_against_reference(dev, fixture, cfg):
    """cfg2 / w64 fp16 mode vs the reference's fp32 output: >= 44 dB and max-abs <= 0.05 (reference under fp16
    autocast: 48.0 dB / 0.021 at cfg2; bf16 mode: 28 dB)."""
    g = golden(fixture)
    net = _net(cfg, int(g["seed"]), dev, "fp16")
    with torch.no_grad():
        out = net(T(g["lq"]).to(dev)).cpu()
    ref = T(g["out"])
    psnr = _psnr(out, ref)
    assert psnr >= 44.0 and (out - ref).abs().max().item() <= 0.05, (psnr, (out - ref).abs().max().item())


def test_fp16_training_step_uses_loss_scaling(dev):
    """fp16 trainer: GradScaler semantics by default (scale 2^16), finite steps, loss close to the fp32 trainer's."""
    from lowlight_image_enhancement_amd.train import NBPTrainer
    cfg = dict(width=32, enc_blk_nums=[1, 1, 1], middle_blk_num=2, dec_blk_nums=[1, 1, 1])
    trs = {}
    gen = torch.Generator(device=dev).manual_seed(11)
    lq, gt = (torch.rand(2, 3, 64, 64, device=dev, generator=gen) for _ in range(2))
    r = torch.ones(2, 1, 1, 1, device=dev)
    for prec in ("fp32", "fp16"):
        tr = NBPTrainer(_net(cfg, 60, dev, prec), w_l1=1.0, w_ssim=0.05, w_phys=0.1)
        for _ in range(3):
            tr.step(lq, gt, lq, r)
        trs[prec] = (tr, tr.logs())
    tr16, logs16 = trs["fp16"]
    assert tr16.scaler is not None and logs16["loss_scale"] == 65536.0 and tr16.skipped_steps == 0
    assert abs(logs16["Total"] - trs["fp32"][1]["Total"]) <= 2e-3 * trs["fp32"][1]["Total"]
    assert abs(logs16["grad_norm"] - trs["fp32"][1]["grad_norm"]) <= 2e-2 * trs["fp32"][1]["grad_norm"]


def test_vgg_full_depth_input_gradient_fp16_vs_bf16(dev):
    """VGG19 features[:36] input gradient (PerceptualLoss backward) vs float64 torch: fp16 under the trainer's loss
    scale must be well under bf16's error (measured 11.6 % vs 32.4 % rel. at full depth, scripts/diag_vgg.py; the rest is
    ReLU-mask / max-pool argmax flips from forward rounding, present in any 16-bit forward)."""
    import torch.nn.functional as Fn
    from lowlight_image_enhancement_amd._lib import call
    from lowlight_image_enhancement_amd.vgg import VGG19_CFG, VGGStack, _layers, input_grad, prep_input
    from lowlight_image_enhancement_amd.vgg import synthetic_state_dict
    sd = synthetic_state_dict(VGG19_CFG, 36, 0)
    sd = {k: (v + 0.01 if k.endswith("bias") else v) for k, v in sd.items()}
    g = torch.Generator().manual_seed(2)
    gen, tgt = torch.rand(2, 3, 64, 48, generator=g), torch.rand(2, 3, 64, 48, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406], dtype=torch.float64).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], dtype=torch.float64).view(1, 3, 1, 1)

    def stack(h):
        for kind, idx, _, _ in _layers(VGG19_CFG, 36):
            h = Fn.max_pool2d(h, 2) if kind == "pool" else Fn.relu(
                Fn.conv2d(h, sd[f"{idx}.weight"].double(), sd[f"{idx}.bias"].double(), padding=1))
        return h

    xr = gen.double().requires_grad_(True)
    Fn.mse_loss(stack((xr - mean) / std), stack((tgt.double() - mean) / std)).backward()
    errs = {}
    for dt, scale in ((1, 1.0), (2, 65536.0)):
        st = VGGStack(VGG19_CFG, 36, dev, sd, dtype=dt)
        fg, tape, _ = st.forward(prep_input(gen.to(dev), dtype=dt), save=True)
        ft, _, _ = st.forward(prep_input(tgt.to(dev), dtype=dt), save=False)
        d = torch.empty_like(fg)
        call("feat_dist_bwd", fg, ft, fg.numel(), 0, 1.0 / fg.numel(), 1, torch.full((1,), scale, device=dev), d, dt)
        errs[dt] = _rel(input_grad(st.backward(tape, d), gen.to(dev)) / scale, xr.grad)
    assert errs[2] < 0.15 and errs[2] < errs[1] / 2.5, errs
