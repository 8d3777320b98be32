"""Every BASELINE.json config under a GPU parity test, plus the public loss classes and the optimizer's step verdict.

* configs[1] (cfg2): the w32 [2,2,4,8]/12/[2,2,2,2] model, rgb B2, bs 2 x 256^2 -- one fused training step (forward,
  L1 + 0.05 SSIM + 0.1 Phys_srgb, backward, clip 0.01, AdamW) against the oracle (per-tensor gradients, losses,
  post-step parameters) and the forward / backward against the reference's own outputs (nafnet_cfg2.npz, made by
  tests/golden/make_golden.py from the reference); bf16 perf mode at a stated PSNR bound.
* configs[2] (cfg3): the same model's loss head with all six HybridLossPlus terms at bs 1 x 512^2 against the oracle
  (synthetic VGG19 / LPIPS weights: the pretrained files are a download; parity unpinned for real weights).
* configs[3] (cfg4): the w64 model (C = 1024 in the middle level) at 2 x 64^2 against the reference's outputs.
* configs[4] (cfg5): phys_cons_raw with expo_ratio in {100, 250, 300}, psnr_linear / ssim_linear at data_range 4095, at
  8 x 3 x 1024^2 (fp32 and fp16 inputs) against the reference's outputs (cfg5_raw.npz).
Tolerances (BASELINE.json north_star): fp32 restored image within 1e-4 max-abs, loss scalars within 1e-5 relative.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from conftest import golden

pytestmark = pytest.mark.gpu
T = torch.from_numpy

CFG2 = dict(width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
CFG4 = dict(width=64, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
BLK = lambda cfg: {k: v for k, v in cfg.items() if k != "width"}  # noqa: E731


def _recipe_net(cfg, seed, dev, precision="fp32"):
    from param_recipe import recipe_state
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    net = create_newbp_net(in_channels=3, kernel_type="rgb", kernel_spec="B2", **cfg)
    sd = recipe_state([(k, tuple(v.shape)) for k, v in net.state_dict().items()], seed)
    net.load_state_dict(sd)
    net = net.to(dev)
    net.precision = precision
    return net, sd


def _psnr(a, b):
    mse = ((a.double() - b.double()) ** 2).mean().item()
    return float("inf") if mse == 0 else 10 * np.log10(1.0 / mse)


def _grads_ref_layout(net, flat_grad):
    return {k: net._to_reference(e, flat_grad[e.offset:e.offset + e.numel]).cpu() for k, e in net.entries.items()}


# ---------------------------------------------------------------------------------------------- configs[1]: cfg2
def test_cfg2_training_step_fp32_against_oracle_and_reference(dev):
    from lowlight_image_enhancement_amd.train import NBPTrainer
    from oracle.train_step import OracleTrainer
    torch.set_num_threads(16)
    g = golden("nafnet_cfg2.npz")
    net, sd = _recipe_net(CFG2, int(g["seed"]), dev)
    lq, gt = T(g["lq"]), T(g["gt"])
    r = torch.ones(2, 1, 1, 1)
    w = dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1)
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", **w)
    out = tr.step(lq.to(dev), gt.to(dev), lq.clamp(0, 1).to(dev), r.to(dev))
    logs = tr.logs()
    # the reference's own forward (same weights, same batch)
    assert (out.cpu() - T(g["out"])).abs().max().item() <= 1e-4
    assert abs(logs["L1_raw"] - float(g["L1"])) <= 1e-5 * float(g["L1"])
    ora = OracleTrainer(sd, BLK(CFG2), **w)
    ref_out, ref_logs = ora.step(lq, gt, lq.clamp(0, 1), r)
    assert (out.cpu() - ref_out.detach()).abs().max().item() <= 1e-4
    for k in ("L1_raw", "SSIM", "Phys", "Total"):
        ref = float(ref_logs[k])
        assert abs(logs[k] - ref) <= 1e-5 * abs(ref), (k, logs[k], ref)
    grads = _grads_ref_layout(net, tr.grad)
    for k, p in ora.P.items():
        scale = p.grad.abs().max().item()
        err = (grads[k] - p.grad).abs().max().item()
        assert err <= 1e-3 * scale + 1e-8, (k, err, scale)
    # one AdamW step: compare where the gradient sign is well defined (Adam's first step is lr * sign(g))
    post = net.state_dict()
    worst = 0.0
    for k, p in ora.P.items():
        m = p.grad.abs() > 1e-3 * p.grad.abs().max()
        if m.any():
            worst = max(worst, (post[k].cpu() - p.detach())[m].abs().max().item())
    assert worst < 5e-6, worst


def test_cfg2_bf16_mode_against_reference(dev):
    """bf16 perf mode (bf16 storage + MFMA operands, fp32 accumulation / statistics) at cfg2 against the reference's
    fp32 output.  With active blocks (beta, gamma ~ N(0, 0.2)) bf16 rounding compounds over the 36 blocks: the
    reference's OWN forward under torch.autocast(bfloat16) reaches only 30.0 dB on this batch (max-abs 0.156; fp16
    autocast: 48.0 dB / 0.021, measured on CPU in the build container).  Here: >= 26 dB, max-abs <= 0.3 (measured
    28.1 dB / 0.206: bf16 storage at more points than autocast).  (The bench's 55 dB is at the reference's zero
    init, where every block is an identity.)"""
    g = golden("nafnet_cfg2.npz")
    net, sd = _recipe_net(CFG2, int(g["seed"]), dev, precision="bf16")
    lq = T(g["lq"])
    with torch.no_grad():
        out = net(lq.to(dev)).cpu()
    ref = T(g["out"])
    psnr = _psnr(out, ref)
    assert psnr >= 26.0 and (out - ref).abs().max().item() <= 0.3, (psnr, (out - ref).abs().max().item())


# ---------------------------------------------------------------------------------------------- configs[3]: cfg4
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_w64_model_against_reference(dev, precision):
    """The cfg4 per-GPU model (w64: C = 512 / 1024 at the deepest levels) against the reference's forward / backward
    (fp32: 1e-4 max-abs output, 1e-5 rel losses, gradient sums / norms; bf16: >= 26 dB, see the cfg2 bf16 test)."""
    from lowlight_image_enhancement_amd.NewBP_model.losses import PhysicalConsistencyLossSRGB, l1_loss
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_crosstalk_psf
    g = golden("nafnet_w64.npz")
    net, _ = _recipe_net(CFG4, int(g["seed"]), dev, precision)
    lq, gt, r = T(g["lq"]).to(dev), T(g["gt"]).to(dev), T(g["ratio"]).to(dev)
    out = net(lq)
    ref = T(g["out"])
    if precision == "bf16":
        psnr = _psnr(out.detach().cpu(), ref)
        assert psnr >= 26.0 and (out.detach().cpu() - ref).abs().max().item() <= 0.3, psnr
        return
    assert (out.detach().cpu() - ref).abs().max().item() <= 1e-4
    L1 = l1_loss(out, gt)
    Lp = PhysicalConsistencyLossSRGB(create_crosstalk_psf("rgb", "B2").to(dev))(out.clamp(0, 1), (lq * r).clamp(0, 1), r)
    (L1 + 0.1 * Lp).backward()
    assert abs(L1.item() - float(g["L1"])) <= 1e-5 * float(g["L1"])
    assert abs(Lp.item() - float(g["Phys"])) <= 1e-5 * float(g["Phys"])
    grads = _grads_ref_layout(net, net.flat.grad)
    for k in [str(k) for k in g["keys"]]:
        ref_s, ref_n = float(g["gsum:" + k]), float(g["gnorm:" + k])
        assert abs(float(grads[k].double().sum()) - ref_s) <= 1e-3 * (abs(ref_s) + ref_n) + 1e-7, k
        assert abs(float(grads[k].double().norm()) - ref_n) <= 1e-3 * ref_n + 1e-7, k


# ---------------------------------------------------------------------------------------------- configs[4]: cfg5
def _cfg5_inputs():
    from synth_inputs import cfg5_inputs
    return cfg5_inputs()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_cfg5_phys_cons_raw_1024(dev, dtype):
    """phys_cons_raw (metrics/phys_consistency.py:260) at 8 x 3 x 1024^2 with exposure ratios from {100, 250, 300}, and
    the data_range = 4095 linear metrics, against the reference's outputs (fp16 inputs are cast to fp32 by the
    metric, :302-303)."""
    from lowlight_image_enhancement_amd.metrics.linear import psnr_linear, ssim_linear
    from lowlight_image_enhancement_amd.metrics.phys_consistency import phys_cons_raw
    g = golden("cfg5_raw.npz")
    pred, obs, ratios, sl, ss = _cfg5_inputs()
    assert sl == int(g["sum_long"]) and ss == int(g["sum_short"])  # the regenerated batch is the fixture's
    P, O = T(pred).to(dev, dtype), T(obs).to(dev, dtype)
    r = T(ratios).to(dev)
    psf = T(g["psf"]).to(dev)
    if dtype == torch.float16:
        got = phys_cons_raw(P, O, psf, r, reduction="none")
        np.testing.assert_allclose(got.cpu().numpy(), g["raw_fp16_none"], rtol=1e-5)
        return
    np.testing.assert_allclose(phys_cons_raw(P, O, psf, r).cpu().numpy(), g["raw_mean"], rtol=1e-5)
    np.testing.assert_allclose(phys_cons_raw(P, O, psf, r, reduction="none").cpu().numpy(), g["raw_none"], rtol=1e-5)
    got = phys_cons_raw(P, O, psf, r, reduction="sum", robust="charbonnier", padding="replicate", crop="same")
    np.testing.assert_allclose(got.cpu().numpy(), g["raw_charb_sum"], rtol=1e-5)
    long12 = P * r.view(-1, 1, 1, 1) * 4095.0
    short12 = O * 4095.0
    np.testing.assert_allclose(psnr_linear(short12, long12, data_range=4095.0, reduction="none").cpu().numpy(),
                               g["psnr4095_none"], rtol=1e-6)
    np.testing.assert_allclose(ssim_linear(short12, long12, data_range=4095.0, reduction="none").cpu().numpy(),
                               g["ssim4095_none"], atol=2e-6)


def test_cfg5_training_step_1024_against_oracle(dev):
    """configs[4]'s per-GPU step at one 1024 x 1024 image: the cfg2 model (active layer scales), one fused training step
    (L1 + 0.05 SSIM + 0.1 Phys_srgb, clip, AdamW) in the fp32 parity mode against the oracle (output 1e-4 max-abs,
    losses 1e-5 rel, per-tensor gradients 1e-3), then phys_cons_raw (phys_consistency.py:260-320) on the restored
    image against the oracle's metric on the oracle's output, for each expo_ratio in {100, 250, 300}, fp32 and fp16
    inputs (fp32 accumulation).  bench.py's `cfg5` line times the same step at 8 images per GPU in fp16."""
    from lowlight_image_enhancement_amd.metrics.phys_consistency import phys_cons_raw
    from lowlight_image_enhancement_amd.train import NBPTrainer
    from oracle.physics import phys_cons
    from oracle.train_step import OracleTrainer
    torch.set_num_threads(16)
    net, sd = _recipe_net(CFG2, 55, dev)
    g = torch.Generator().manual_seed(5)
    lq, gt = torch.rand(1, 3, 1024, 1024, generator=g), torch.rand(1, 3, 1024, 1024, generator=g)
    r = torch.ones(1, 1, 1, 1)
    w = dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1)
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", **w)
    out = tr.step(lq.to(dev), gt.to(dev), lq.clamp(0, 1).to(dev), r.to(dev)).detach()
    logs = tr.logs()
    ora = OracleTrainer(sd, BLK(CFG2), **w)
    ref_out, ref_logs = ora.step(lq, gt, lq.clamp(0, 1), r)
    ref_out = ref_out.detach()
    assert (out.cpu() - ref_out).abs().max().item() <= 1e-4
    for k in ("L1_raw", "SSIM", "Phys", "Total"):
        ref = float(ref_logs[k])
        assert abs(logs[k] - ref) <= 1e-5 * abs(ref), (k, logs[k], ref)
    grads = _grads_ref_layout(net, tr.grad)
    for k, p in ora.P.items():
        scale = p.grad.abs().max().item()
        assert (grads[k] - p.grad).abs().max().item() <= 1e-3 * scale + 1e-8, k
    psf = T(golden("cfg5_raw.npz")["psf"])  # the reference's [C_out, C_in, 3, 3] PSF of the cfg5 fixture
    for ratio in (100.0, 250.0, 300.0):
        rr = torch.full((1,), ratio)
        for dt in (torch.float32, torch.float16):
            got = phys_cons_raw(out.clamp_min(0).to(dt), lq.to(dev, dt), psf.to(dev), rr.to(dev))
            ref = phys_cons(ref_out.clamp_min(0).to(dt), lq.to(dt), psf, rr, clamp01=False)
            assert abs(float(got) - float(ref)) <= 1e-5 * abs(float(ref)), (ratio, dt, float(got), float(ref))


# ---------------------------------------------------------------------------------------------- configs[2]: cfg3
def _synthetic_loss_weights():
    from lowlight_image_enhancement_amd.lpips import TAP_CH
    from lowlight_image_enhancement_amd.vgg import VGG16_CFG, VGG19_CFG, synthetic_state_dict
    v19 = synthetic_state_dict(VGG19_CFG, 36, seed=0)
    v16 = synthetic_state_dict(VGG16_CFG, 30, seed=0)
    gl = torch.Generator().manual_seed(0)
    lins = [(torch.randn(c, generator=gl) * 0.1).abs() for c in TAP_CH]
    return v19, v16, lins


def test_cfg3_loss_head_512_against_oracle(dev):
    """cfg3: cfg2 model + every HybridLossPlus term (L1, VGG19 Perc, LPIPS(vgg), ΔE00, SSIM, Phys_srgb) at bs 1 x 512^2,
    fp32 network mode, against the oracle with the same synthetic VGG weights.  The fp32 mode runs the VGG / LPIPS
    trunks in fp32 like the reference (NewBP_model/losses.py:63-69): every loss scalar within 1e-5 rel; the parameter
    gradient within 1e-3 rel-norm and per tensor within 3e-3 of the tensor's max (fp32 max-pool near-ties in the
    trunks; the cfg2 step without them meets 1e-3 per tensor)."""
    from lowlight_image_enhancement_amd.NewBP_model.losses import PerceptualLoss
    from lowlight_image_enhancement_amd.lpips import LPIPS
    from lowlight_image_enhancement_amd.train import NBPTrainer
    from oracle.train_step import OracleTrainer
    torch.set_num_threads(16)
    net, sd = _recipe_net(CFG2, 310, dev)
    v19, v16, lins = _synthetic_loss_weights()
    lp_sd = {f"net.slice1.{k}": v for k, v in v16.items()}
    lp_sd.update({f"lin{k}.model.1.weight": w.view(1, -1, 1, 1) for k, w in enumerate(lins)})
    w = dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_perc=0.02, w_lpips=0.05, w_deltaE=0.02)
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", perceptual=PerceptualLoss(device=dev, weights=v19),
                    lpips=LPIPS(net="vgg", weights=lp_sd), **w)
    assert tr.vgg_dt == 0
    gen = torch.Generator().manual_seed(311)
    lq, gt = torch.rand(1, 3, 512, 512, generator=gen), torch.rand(1, 3, 512, 512, generator=gen)
    r = torch.ones(1, 1, 1, 1)
    tr.loss_and_grad(lq.to(dev), gt.to(dev), lq.to(dev), r.to(dev))
    logs = tr.logs()
    ora = OracleTrainer(sd, BLK(CFG2), w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_de=0.02, w_perc=0.02, w_lpips=0.05,
                        vgg19_sd=v19, lpips_parts=(v16, lins))
    _, tot, ref_logs = ora.loss(lq, gt, lq, r)
    tot.backward()
    for k in ("L1_raw", "SSIM", "Phys", "DeltaE", "Perc", "LPIPS", "Total"):
        ref = float(ref_logs[k])
        assert abs(logs[k] - ref) <= 1e-5 * abs(ref), (k, logs[k], ref)
    grads = _grads_ref_layout(net, tr.grad)
    num = sum(((grads[k] - p.grad) ** 2).sum().item() for k, p in ora.P.items())
    den = sum((p.grad ** 2).sum().item() for p in ora.P.values())
    assert (num / den) ** 0.5 < 1e-3, (num / den) ** 0.5
    for k, p in ora.P.items():  # measured worst 1.8e-3 of the tensor's max (encoders.0.0.conv1.weight): max-pool
        scale = p.grad.abs().max().item()  # near-ties in the VGG / LPIPS trunks (tests/test_gpu_vgg.py)
        err = (grads[k] - p.grad).abs().max().item()
        assert err <= 3e-3 * scale + 1e-8, (k, err, scale)


def test_cfg3_loss_head_fp16_trunk(dev):
    """The fp16 mode's loss head (fp16 network and fp16 VGG / LPIPS trunks under the dynamic loss scale, the
    reference's autocast counterpart) at a stated bound against the fp32 oracle: Perc / LPIPS within 3 %, the pixel
    terms within 1e-2 (fp16 network output)."""
    from lowlight_image_enhancement_amd.NewBP_model.losses import PerceptualLoss
    from lowlight_image_enhancement_amd.lpips import LPIPS
    from lowlight_image_enhancement_amd.train import NBPTrainer
    from oracle.train_step import OracleTrainer
    torch.set_num_threads(16)
    net, sd = _recipe_net(CFG2, 312, dev, "fp16")
    v19, v16, lins = _synthetic_loss_weights()
    lp_sd = {f"net.slice1.{k}": v for k, v in v16.items()}
    lp_sd.update({f"lin{k}.model.1.weight": w.view(1, -1, 1, 1) for k, w in enumerate(lins)})
    w = dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_perc=0.02, w_lpips=0.05, w_deltaE=0.02)
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", perceptual=PerceptualLoss(device=dev, weights=v19),
                    lpips=LPIPS(net="vgg", weights=lp_sd), **w)
    assert tr.vgg_dt == 2
    gen = torch.Generator().manual_seed(313)
    lq, gt = torch.rand(1, 3, 256, 256, generator=gen), torch.rand(1, 3, 256, 256, generator=gen)
    r = torch.ones(1, 1, 1, 1)
    tr.loss_and_grad(lq.to(dev), gt.to(dev), lq.to(dev), r.to(dev))
    logs = tr.logs()
    ora = OracleTrainer(sd, BLK(CFG2), w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_de=0.02, w_perc=0.02, w_lpips=0.05,
                        vgg19_sd=v19, lpips_parts=(v16, lins))
    with torch.no_grad():
        _, _, ref_logs = ora.loss(lq, gt, lq, r)
    for k in ("L1_raw", "SSIM", "Phys", "DeltaE"):
        ref = float(ref_logs[k])
        assert abs(logs[k] - ref) <= 1e-2 * abs(ref), (k, logs[k], ref)
    for k in ("Perc", "LPIPS"):
        ref = float(ref_logs[k])
        assert abs(logs[k] - ref) <= 3e-2 * abs(ref), (k, logs[k], ref)


# ---------------------------------------------------------------------------------------------- public loss classes
def _hybrid_kwargs():
    """configs/colab/sid_newbp_rgb.yml:80-96 hybrid_opt, as image_restoration_model.py:76-101 turns it into kwargs."""
    return dict(w_l1_raw=1.0, w_perc=0.02, w_lpips=0.05, w_deltaE=0.02, w_ssim=0.0, w_phys=0.1, use_deltaE=True,
                use_ssim=False, use_lpips=False, use_phys=True, use_uncertainty=False)


def test_hybrid_loss_plus_from_rgb_config(dev):
    """HybridLossPlus built exactly as ImageRestorationModel.init_training_settings does from the rgb config, called
    as optimize_parameters calls it (:293-301): term values, log keys and d total / d output vs the oracle."""
    import oracle.losses as OL
    import oracle.physics as OP
    from lowlight_image_enhancement_amd.NewBP_model.losses import HybridLossPlus
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_crosstalk_psf
    v19, _, _ = _synthetic_loss_weights()
    kw = _hybrid_kwargs()
    kw["device"] = "cuda"
    kw["physics_psf_module"] = create_crosstalk_psf(psf_mode="rgb", kernel_spec="B2")
    crit = HybridLossPlus(**kw).to(dev)
    gen = torch.Generator().manual_seed(40)
    out = torch.rand(2, 3, 64, 48, generator=gen) * 1.2 - 0.1
    gt, lq = torch.rand(2, 3, 64, 48, generator=gen), torch.rand(2, 3, 64, 48, generator=gen)
    ratio = torch.tensor([1.0, 2.0]).view(2, 1, 1, 1)
    short = (lq * ratio).clamp(0, 1)
    o = out.to(dev).requires_grad_(True)
    total, logs = crit(Bhat_raw=o, B_raw=gt.to(dev), A_raw=lq.to(dev), expo_ratio=ratio.to(dev),
                       Bhat_srgb01=o.clamp(0.0, 1.0), B_srgb01=gt.to(dev).clamp(0.0, 1.0),
                       A_srgb01=short.to(dev).clamp(0.0, 1.0))
    total.backward()
    assert list(logs) == ["L1_raw", "Perc", "DeltaE", "Phys", "Total"]  # the reference's keys for this config
    orr = out.clone().requires_grad_(True)
    k = OP.normalize_psf(OP.build_psf_kernels("rgb", "B2"))
    terms = dict(L1_raw=OL.l1(orr, gt), Perc=OL.perceptual_loss(v19, orr.clamp(0, 1), gt.clamp(0, 1)),
                 DeltaE=OL.deltae00_loss(orr.clamp(0, 1), gt.clamp(0, 1)),
                 Phys=OP.phys_srgb_loss(orr.clamp(0, 1), short.clamp(0, 1), ratio, k))
    wts = dict(L1_raw=1.0, Perc=0.02, DeltaE=0.02, Phys=0.1)
    ref_total = sum(wts[n] * v for n, v in terms.items())
    ref_total.backward()
    for n, v in terms.items():  # the VGG trunk runs fp32 outside autocast, as the reference's does
        assert abs(logs[n].item() - v.item()) <= 1e-5 * abs(v.item()), (n, logs[n].item(), v.item())
    assert abs(logs["Total"].item() - ref_total.item()) <= 1e-5 * ref_total.item()
    a, b = o.grad.cpu().double().flatten(), orr.grad.double().flatten()
    assert ((a - b).norm() / b.norm()).item() < 1e-5


def test_hybrid_loss_plus_zero_weight_terms_still_logged(dev):
    """The reference always evaluates Perc (losses.py:337) and ΔE (use_deltaE): weight 0 keeps their log keys."""
    from lowlight_image_enhancement_amd.NewBP_model.losses import HybridLossPlus
    crit = HybridLossPlus(device="cuda", w_perc=0.0, w_deltaE=0.0, use_ssim=False, use_phys=False).to(dev)
    gen = torch.Generator().manual_seed(41)
    a, b = (torch.rand(1, 3, 32, 32, generator=gen).to(dev) for _ in range(2))
    x = a.clone().requires_grad_(True)
    total, logs = crit(Bhat_raw=x, B_raw=b, A_raw=b, expo_ratio=torch.ones(1, device=dev), Bhat_srgb01=x.clamp(0, 1),
                       B_srgb01=b)
    assert list(logs) == ["L1_raw", "Perc", "DeltaE", "Total"]
    assert logs["Perc"].item() > 0 and logs["DeltaE"].item() > 0
    total.backward()
    assert abs(total.item() - logs["L1_raw"].item()) <= 1e-7


def test_hybrid_loss_value_and_gradient(dev):
    """HybridLoss(lambda_l1, lambda_perceptual, device) (losses.py:72-89): (total, l1, perc) and d total / d gen."""
    import oracle.losses as OL
    from lowlight_image_enhancement_amd.NewBP_model.losses import HybridLoss
    v19, _, _ = _synthetic_loss_weights()
    crit = HybridLoss(lambda_l1=1.0, lambda_perceptual=0.1, device="cuda")
    gen = torch.Generator().manual_seed(42)
    x, y = torch.rand(2, 3, 48, 40, generator=gen), torch.rand(2, 3, 48, 40, generator=gen)
    xd = x.to(dev).requires_grad_(True)
    total, l1, perc = crit(xd, y.to(dev))
    total.backward()
    xr = x.clone().requires_grad_(True)
    rl1, rperc = OL.l1(xr, y), OL.perceptual_loss(v19, xr, y)
    (rl1 + 0.1 * rperc).backward()
    assert abs(l1.item() - rl1.item()) <= 1e-5 * rl1.item()
    assert abs(perc.item() - rperc.item()) <= 1e-5 * rperc.item()
    assert abs(total.item() - (l1.item() + 0.1 * perc.item())) <= 1e-6
    a, b = xd.grad.cpu().double().flatten(), xr.grad.double().flatten()
    assert ((a - b).norm() / b.norm()).item() < 1e-5


@pytest.mark.parametrize("kernel_type,spec", [("panchromatic", "P2"), ("rgb", "B2")])
def test_newbp_function_forward_and_adjoint(dev, kernel_type, spec):
    """NewBPFunction through NewBPLayer(deprecated=False): conv2d forward, conv_transpose2d backward with the
    un-normalised kernel (newbp_layer.py:7-21, 44-85; adjoint pinned by core_tests/test_physics_loss_grad.py:65-86)."""
    from lowlight_image_enhancement_amd.NewBP_model.newbp_layer import NewBPLayer
    layer = NewBPLayer(3, kernel_type, spec, deprecated=False).to(dev)
    gen = torch.Generator().manual_seed(43)
    x, gy = torch.rand(2, 3, 33, 47, generator=gen), torch.randn(2, 3, 33, 47, generator=gen)
    xd = x.to(dev).requires_grad_(True)
    y = layer(xd)
    y.backward(gy.to(dev))
    k = layer.kernel.detach().cpu().double()
    ref = Fn.conv2d(x.double(), k, padding=1, groups=3)
    assert (y.detach().cpu().double() - ref).abs().max().item() <= 1e-6
    adj = Fn.conv_transpose2d(gy.double(), k, padding=1, groups=3)
    assert (xd.grad.cpu().double() - adj).abs().max().item() <= 1e-6
    with pytest.raises(RuntimeError):
        NewBPLayer(3, kernel_type, spec)(xd)


# ---------------------------------------------------------------------------------------------- step verdict
def _small_trainer(dev, precision="fp32", **kw):
    from lowlight_image_enhancement_amd.train import NBPTrainer
    net, _ = _recipe_net(dict(width=16, enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1]), 50, dev,
                         precision)
    return NBPTrainer(net, psf_mode="rgb", psf_spec="B2", w_l1=1.0, w_ssim=0.05, w_phys=0.1, **kw)


def _batch(dev, seed, nan=False):
    gen = torch.Generator(device=dev).manual_seed(seed)
    lq, gt = (torch.rand(2, 3, 32, 32, device=dev, generator=gen) for _ in range(2))
    if nan:
        lq[1, 2, 5, 7] = float("nan")
    return lq, gt, lq.clamp(0, 1), torch.ones(2, 1, 1, 1, device=dev)


@pytest.mark.parametrize("precision,graph", [("fp32", False), ("bf16", False), ("fp32", True), ("bf16", True)])
def test_nonfinite_step_is_skipped(dev, precision, graph):
    """A batch that makes the gradient non-finite must leave parameters and AdamW moments untouched (GradScaler's
    scaler.step skip, image_restoration_model.py:314), count as skipped, and not advance AdamW's step count."""
    tr = _small_trainer(dev, precision)
    run = tr.graph_step if graph else tr.step
    run(*_batch(dev, 1))
    tr.logs()
    snap = [x.clone() for x in (tr.net.flat.data, tr.exp_avg, tr.exp_avg_sq)]
    run(*_batch(dev, 2, nan=True))
    for a, b in zip(snap, (tr.net.flat.data, tr.exp_avg, tr.exp_avg_sq)):
        assert torch.equal(a, b)
    assert tr.t == 1 and tr.skipped_steps == 1
    with pytest.raises(RuntimeError):
        tr.logs()  # the loss itself is non-finite: the reference's _ensure_finite raises
    run(*_batch(dev, 3))
    assert tr.t == 2 and not torch.equal(snap[0], tr.net.flat.data)
    assert np.isfinite(tr.logs()["Total"])


def test_skip_between_logs_is_reported_without_a_scaler(dev):
    """without a loss scaler a skipped (non-finite-gradient) step anywhere between two logs() calls must
    raise at the next logs(), not only when it was the last step (the clean step after it hides it from the per-step
    verdict)."""
    tr = _small_trainer(dev, "fp32")
    tr.step(*_batch(dev, 1))
    tr.logs()
    tr.step(*_batch(dev, 2, nan=True))  # skipped
    assert tr.skipped_steps == 1
    tr.step(*_batch(dev, 3))  # clean: the last step alone would not show the skip
    with pytest.raises(RuntimeError, match="non-finite"):
        tr.logs()
    tr.step(*_batch(dev, 4))
    assert np.isfinite(tr.logs()["Total"])  # each skip is reported once


def test_dynamic_loss_scale_is_exact_and_follows_gradscaler(dev):
    """Loss scaling by a power of two commutes with every (linear) backward op, so a dynamically scaled fp32 run
    equals the unscaled one bit for bit; the scale follows torch.amp.GradScaler.update (backoff 0.5 on a skipped
    step, growth 2 after growth_interval finite steps)."""
    a = _small_trainer(dev, "fp32", loss_scale=None)
    b = _small_trainer(dev, "fp32", loss_scale="dynamic", growth_interval=2)
    for s in (1, 2):
        a.step(*_batch(dev, s))
        b.step(*_batch(dev, s))
    assert torch.equal(a.net.flat.data, b.net.flat.data) and torch.equal(a.exp_avg_sq, b.exp_avg_sq)
    assert b.logs()["loss_scale"] == 65536.0 and float(b.scaler[0]) == 131072.0  # grew after 2 finite steps
    b.step(*_batch(dev, 3, nan=True))
    assert float(b.scaler[0]) == 65536.0 and b.skipped_steps == 1 and b.t == 2
