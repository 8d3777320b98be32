"""Pin the CPU oracle against fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import json
import os
import warnings

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from oracle import losses as L
from oracle import nafnet as N
from oracle import physics as P
from oracle.train_step import OracleTrainer

T = torch.from_numpy


def close(a, b, atol=1e-6, rtol=1e-5):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), atol=atol, rtol=rtol)


def test_psf_kernels_bit_exact():
    g = golden("psf.npz")
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        raw = P.build_psf_kernels(mode, spec)
        assert np.array_equal(raw.numpy().view(np.uint32), g[f"{mode}_{spec}_raw"].view(np.uint32))
        k = P.normalize_psf(raw)
        assert np.array_equal(k.numpy().view(np.uint32), g[f"{mode}_{spec}_kernel"].view(np.uint32))
    for t in ("t_mono", "t_rgb", "t_raw"):
        k = P.normalize_psf(T(g[t + "_in"]))
        assert np.array_equal(k.numpy().view(np.uint32), g[t + "_norm"].view(np.uint32))
    with pytest.raises(ValueError):
        P.build_psf_kernels("mono", "B2")
    with pytest.raises(ValueError):
        P.build_psf_kernels("rgb", "P2")
    with pytest.raises(ValueError):
        P.build_psf_kernels("cmy")


def test_psf_conv_fwd_bwd():
    g = golden("psf.npz")
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        k = P.normalize_psf(P.build_psf_kernels(mode, spec))
        x = T(g["x"]).clone().requires_grad_(True)
        y = P.psf_apply(x, k)
        y.backward(T(g["gy"]))
        close(y, g[f"y_{mode}"])
        close(x.grad, g[f"dx_{mode}"])


def test_phys_srgb_all_ratio_forms():
    g = golden("phys_srgb.npz")
    ratios = {"float1": 1.0, "float07": 0.7, "t0d": torch.tensor(1.3), "t1d": torch.tensor([0.6, 1.0, 1.7]),
              "t4d": torch.tensor([0.9, 1.2, 2.5]).view(3, 1, 1, 1)}
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        k = P.normalize_psf(P.build_psf_kernels(mode, spec))
        for rk, r in ratios.items():
            b = T(g["bhat"]).clone().requires_grad_(True)
            loss = P.phys_srgb_loss(b, T(g["a"]), r, k)
            loss.backward()
            close(loss, g[f"{mode}_{rk}_loss"], atol=1e-7)
            close(b.grad, g[f"{mode}_{rk}_grad"], atol=1e-9)
            close(P.align_exposure_srgb(T(g["a"]), r), g[f"{mode}_{rk}_align"], atol=0)
    for name, (mode, spec) in (("mono", ("mono", "P2")), ("rgb", ("rgb", "B2"))):
        k = P.build_psf_kernels(mode, spec)
        for c in (True, False):
            b = T(g["bhat"]).clone().requires_grad_(True)
            loss = P.phys_raw_loss(b, T(g["araw"]), T(g["raw_ratio"]), k, clamp_align=c)
            loss.backward()
            close(loss, g[f"raw_{name}_c{int(c)}_loss"], atol=1e-7)
            close(b.grad, g[f"raw_{name}_c{int(c)}_grad"], atol=1e-9)


def test_phys_raw_groups1_fixtures():
    """The oracle's raw physics loss in the reference's groups == 1 branch (losses.py:182-191) vs the reference's
    outputs: expanded [Co,1,kh,kw] and full [Co,C,kh,kw] kernels, F.l1_loss's channel broadcast, rejected forms."""
    g = golden("phys_raw_full.npz")
    for name in g["cases"]:
        name = str(name)
        b = T(g[f"{name}_bhat"]).clone().requires_grad_(True)
        args = (T(g[f"{name}_a"]), T(g["ratio"]), T(g[f"{name}_k"]))
        if int(g[f"{name}_raises"]):
            with pytest.raises(RuntimeError):
                P.phys_raw_loss(b, *args, clamp_align=bool(g[f"{name}_clamp"]))
            continue
        loss = P.phys_raw_loss(b, *args, clamp_align=bool(g[f"{name}_clamp"]))
        loss.backward()
        close(loss, g[f"{name}_loss"], atol=1e-6)
        close(b.grad, g[f"{name}_grad"], atol=1e-9)


def test_ssim_alignment_helpers_fixtures():
    """The oracle's calculate_ssim input alignment vs the reference's own helpers (metrics/ssim.py:119-167)."""
    import oracle.losses as OL
    g = golden("ssim_align.npz")
    assert torch.equal(OL.luma_bt601(T(g["rgb"])), T(g["luma"]))
    ct, cp = OL.ssim_align_pair(T(g["tgt"]), T(g["pred"]), "center_crop")
    assert torch.equal(ct, T(g["crop_t"])) and torch.equal(cp, T(g["crop_p"]))
    for mode in ("bilinear", "bicubic"):
        assert torch.equal(OL.ssim_align_pair(T(g["tgt"]), T(g["pred"]), "resize", mode)[1], T(g[f"resize_{mode}"]))
        assert torch.equal(OL.ssim_align_pair(T(g["tgt"]), T(g["small"]), "resize", mode)[1], T(g[f"up_{mode}"]))


def test_phys_cons_variant_matrix():
    g = golden("phys_cons.npz")
    cases = json.load(open(os.path.join(GOLDEN, "phys_cons_cases.json")))
    assert len(cases) > 100
    for name in cases:
        fn, padding, crop, robust, rk, psfk, nn_ = name.split("|")
        r = g[f"ratio_{rk}"]
        r = float(r) if r.ndim == 0 else T(r)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            m, amap = P.phys_cons(T(g["pred"]), T(g["obs"]), T(g[psfk]), r, clamp01=(fn == "srgb"), padding=padding,
                                  crop=crop, robust=robust, enforce_nonnegative=bool(int(nn_)), return_map=True,
                                  reduction="none", eps=1e-3 if robust == "charbonnier" else 1e-12)
        close(m, g["v:" + name], atol=1e-6)
        close(amap, g["m:" + name], atol=1e-6)
    for red in ("mean", "sum"):
        close(P.phys_cons(T(g["pred"]), T(g["obs"]), T(g["psf3"]), 1.4, clamp01=False, reduction=red),
              g[f"srgb_noclamp_{red}"])
        close(P.phys_cons(T(g["pred"]), T(g["obs"]), T(g["psf3"]), 0.9, clamp01=False, normalize_psf=False,
                          reduction=red), g[f"raw_nonorm_{red}"])


def test_layernorm2d():
    g = golden("layernorm.npz")
    x = T(g["x"]).clone().requires_grad_(True)
    w = T(g["w"]).clone().requires_grad_(True)
    b = T(g["b"]).clone().requires_grad_(True)
    y = N.layer_norm2d(x, w, b)
    y.backward(T(g["dy"]))
    close(y, g["y"])
    close(x.grad, g["dx"], atol=1e-5)
    close(w.grad, g["dw"], atol=1e-5)
    close(b.grad, g["db"], atol=1e-5)


def test_nafblock():
    g = golden("nafblock.npz")
    Pm = {k[2:]: T(g[k]).clone().requires_grad_(True) for k in g.files if k.startswith("p:")}
    x = T(g["x"]).clone().requires_grad_(True)
    y = N.nafblock(Pm, "", x)
    y.backward(T(g["dy"]))
    close(y, g["y"], atol=1e-5)
    close(x.grad, g["dx"], atol=1e-5)
    for k, p in Pm.items():
        close(p.grad, g["g:" + k], atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("name,cfg,mode", [
    ("nafnet_cfg0.npz", dict(enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1]), ("rgb", "B2")),
    ("nafnet_cfg0_pad.npz", dict(enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1]), ("mono", "P2")),
])
def test_nafnet_full(name, cfg, mode):
    g = golden(name)
    keys = [str(k) for k in g["keys"]]
    shapes = N.nafnet_param_shapes(width=8, **cfg)
    assert [k for k, _ in shapes] == keys
    Pm = {k: T(g["p:" + k]).clone().requires_grad_(True) for k in keys}
    out = N.nafnet(Pm, T(g["lq"]), **cfg)
    close(out, g["out"], atol=2e-5)
    k = P.normalize_psf(P.build_psf_kernels(*mode))
    r = T(g["ratio"])
    short = (T(g["lq"]) * r).clamp(0, 1)
    l1 = L.l1(out, T(g["gt"]))
    ph = P.phys_srgb_loss(out.clamp(0, 1), short, r, k)
    (l1 + 0.1 * ph).backward()
    close(l1, g["L1"], atol=1e-6)
    close(ph, g["Phys"], atol=1e-6)
    for kk in keys:
        close(Pm[kk].grad, g["g:" + kk], atol=1e-5, rtol=1e-3)


def test_nafnet_cfg1_by_recipe():
    from param_recipe import recipe_state
    g = golden("nafnet_cfg1.npz")
    cfg = dict(enc_blk_nums=[1, 1, 1, 1], middle_blk_num=1, dec_blk_nums=[1, 1, 1, 1])
    shapes = N.nafnet_param_shapes(width=16, **cfg)
    Pm = {k: v.requires_grad_(True) for k, v in recipe_state(shapes, int(g["seed"])).items()}
    assert sum(v.numel() for v in Pm.values()) == int(g["nparams"])
    out = N.nafnet(Pm, T(g["lq"]), **cfg)
    close(out, g["out"], atol=3e-5)
    k = P.normalize_psf(P.build_psf_kernels("mono", "P2"))
    l1 = L.l1(out, T(g["gt"]))
    ph = P.phys_srgb_loss(out.clamp(0, 1), (T(g["lq"])).clamp(0, 1), T(g["ratio"]), k)
    (l1 + 0.1 * ph).backward()
    close(l1, g["L1"], atol=1e-6)
    close(ph, g["Phys"], atol=1e-6)
    for kk, p in Pm.items():
        close(p.grad.double().sum(), g["gsum:" + kk], atol=1e-5, rtol=1e-3)


def test_train_steps_cfg0():
    g = golden("train_steps_cfg0.npz")
    cfg = dict(enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1])
    keys = [k for k, _ in N.nafnet_param_shapes(width=8, **cfg)]
    tr = OracleTrainer({k: T(g["init:" + k]) for k in keys}, cfg, w_l1=1.0, w_phys=0.1)
    for s in range(2):
        lq, gt = T(g[f"s{s}:lq"]), T(g[f"s{s}:gt"])
        ratio = torch.ones(2, 1, 1, 1)
        _, logs = tr.step(lq, gt, (lq * ratio).clamp(0, 1), ratio)
        close(logs["L1_raw"], g[f"s{s}:L1"], atol=1e-6)
        close(logs["Phys"], g[f"s{s}:Phys"], atol=1e-6)
        close(logs["Total"], g[f"s{s}:total"], atol=1e-6)
        close(logs["gradnorm"], g[f"s{s}:gradnorm"], rtol=1e-5)
        for k in keys:
            close(tr.P[k], g[f"s{s}:p:{k}"], atol=2e-7, rtol=1e-5)


def test_ciede2000_forms():
    g = golden("ciede2000.npz")
    close(L.ciede2000_loss_form(T(g["lab1"]), T(g["lab2"])), g["loss_sharma"], atol=2e-5)
    close(L.ciede2000_loss_form(T(g["rl1"]), T(g["rl2"])), g["loss_rand"], atol=5e-5, rtol=1e-5)
    close(L.deltae00_metric_map(T(g["lab1"]), T(g["lab2"])), g["met_sharma"], atol=2e-5)
    close(L.deltae00_metric_map(T(g["rl1"]), T(g["rl2"])), g["met_rand"], atol=5e-5, rtol=1e-5)
    # the reference's own Sharma KAT tolerance (standard_tests/test_color_error.py:161-197): 1.5
    assert np.abs(g["met_sharma"].ravel() - g["sharma_gold"]).max() < 1.5
    li = T(g["rl1"]).clone().requires_grad_(True)
    L.ciede2000_loss_form(li, T(g["rl2"])).mean().backward()
    close(li.grad, g["loss_rand_grad"], atol=1e-6, rtol=1e-4)


def test_linear_metrics():
    g = golden("linear_metrics.npz")
    a, b = T(g["a"]), T(g["b"])
    close(L.psnr_linear(b, a, reduction="none"), g["psnr_none"], rtol=1e-10)
    close(L.psnr_linear(b, a), g["psnr_mean"], rtol=1e-10)
    close(L.psnr_linear(b * 4095, a * 4095, data_range=4095.0, reduction="none"), g["psnr_4095"], rtol=1e-6)
    close(L.ssim_linear(b, a, reduction="none"), g["ssim_none"], atol=1e-6)
    close(L.ssim_linear(b, a, reduction="none", channel_aggregate="none"), g["ssim_chan"], atol=1e-6)
    assert abs(L.calculate_psnr(a, b, 1.0) - float(g["calc_psnr"])) < 1e-9


def test_ssim_loss_partially_pinned_by_ssim_linear():
    """kornia is absent (parity unpinned for SSIMLoss itself); on inputs whose local variances stay
    positive, kornia's loss equals (1 - ssim_linear)/2 up to window rounding (metrics/linear.py:218-324)."""
    g = golden("linear_metrics.npz")
    a, b = T(g["a"]), T(g["b"])
    ref = (1.0 - float(g["ssim_mean"])) / 2.0
    assert abs(float(L.ssim_loss(b, a)) - ref) < 2e-6
