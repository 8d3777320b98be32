"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Test infrastructure only.  Runs in the build container (where /root/reference is
mounted read-only); the GPU box never runs this script, it only reads the .npz /
.json outputs.  The reference is pure Python and is imported with the stub recipe
of SURVEY.md §8c: `basicsr`, `basicsr.utils` (get_root_logger only),
`basicsr.models`, `basicsr.models.archs` are stub modules, the three arch files
(arch_util.py, local_arch.py, NAFNet_arch.py) are loaded by file path, and
`torchvision` is a stub with an empty `models` namespace (VGG19 weights are a
network download and are never constructed here).

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import logging
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from param_recipe import recipe_state  # noqa: E402
from synth_inputs import cfg5_inputs  # noqa: E402


def load_reference(ref: str):
    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__path__ = []  # mark as package
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    stub("basicsr")
    stub("basicsr.utils", get_root_logger=lambda *a, **k: logging.getLogger("basicsr"))
    stub("basicsr.models")
    stub("basicsr.models.archs")
    arch_dir = os.path.join(ref, "NAFNet_base", "basicsr", "models", "archs")
    for mod in ("arch_util", "local_arch", "NAFNet_arch"):
        full = f"basicsr.models.archs.{mod}"
        spec = importlib.util.spec_from_file_location(full, os.path.join(arch_dir, mod + ".py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[full] = m
        spec.loader.exec_module(m)
    tv = stub("torchvision")
    tv.models = types.SimpleNamespace()
    sys.path.insert(0, ref)
    import NewBP_model.newbp_layer as nl
    import NewBP_model.newbp_net_arch as na
    import NewBP_model.losses as nlo
    import metrics.phys_consistency as pc
    import metrics.linear as lin
    import metrics.psnr as psnr
    import metrics.color_error as ce
    arch = sys.modules["basicsr.models.archs.NAFNet_arch"]
    au = sys.modules["basicsr.models.archs.arch_util"]
    return types.SimpleNamespace(nl=nl, na=na, lo=nlo, pc=pc, lin=lin, psnr=psnr, ce=ce, arch=arch, au=au)


def t2n(t):
    return t.detach().cpu().clone().numpy()


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v if isinstance(v, np.ndarray) else np.asarray(v)) for k, v in arrays.items()})
    print("wrote", path, sum(np.asarray(v).nbytes for v in arrays.values()), "bytes raw")


# ---------------------------------------------------------------------------
def gen_psf(R):
    out = {}
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        psf = R.na.create_crosstalk_psf(mode, spec)
        out[f"{mode}_{spec}_kernel"] = t2n(psf.kernel)
        raw = R.nl.build_psf_kernels(mode, spec)
        out[f"{mode}_{spec}_raw"] = t2n(raw)
        out[f"{mode}_{spec}_sum"] = t2n(raw.view(raw.shape[0], -1).sum(dim=1))
    # the kernels the reference tests construct (core_tests/test_psf_depthwise_and_kernels.py:38-91)
    tk = {
        "t_mono": torch.tensor([[[[0.0, 0.05, 0.0], [0.05, 0.80, 0.05], [0.0, 0.05, 0.0]]]]),
        "t_rgb": torch.cat([
            torch.tensor([[[[0, 0, 0], [0, 1, 0], [0, 0, 0]]]], dtype=torch.float32),
            torch.tensor([[[[0, 1, 0], [1, 2, 1], [0, 1, 0]]]], dtype=torch.float32) / 6.0,
            torch.tensor([[[[1, 0, 1], [0, 1, 0], [1, 0, 1]]]], dtype=torch.float32) / 5.0]),
        "t_raw": torch.tensor([[[[0.0, 1.0, 0.0], [1.0, 6.0, 1.0], [0.0, 1.0, 0.0]]]]),
    }
    for k, v in tk.items():
        out[k + "_in"] = t2n(v)
        out[k + "_norm"] = t2n(R.nl.CrosstalkPSF("mono" if v.shape[0] == 1 else "rgb", v).kernel)
    # forward + backward of CrosstalkPSF (F.conv2d groups=3 zero pad, newbp_layer.py:109-126)
    g = torch.Generator().manual_seed(11)
    x = torch.rand(2, 3, 17, 19, generator=g)
    gy = torch.randn(2, 3, 17, 19, generator=g)
    out["x"] = t2n(x)
    out["gy"] = t2n(gy)
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        psf = R.na.create_crosstalk_psf(mode, spec)
        xi = x.clone().requires_grad_(True)
        y = psf(xi)
        y.backward(gy)
        out[f"y_{mode}"] = t2n(y)
        out[f"dx_{mode}"] = t2n(xi.grad)
    save("psf.npz", **out)


def gen_phys_srgb(R):
    """PhysicalConsistencyLossSRGB (losses.py:206-220) with every ratio form of align_exposure_srgb (:195-203)."""
    g = torch.Generator().manual_seed(12)
    B, H, W = 3, 16, 20
    bhat = torch.rand(B, 3, H, W, generator=g) * 1.1 - 0.05
    a = torch.rand(B, 3, H, W, generator=g) * 0.8
    out = {"bhat": t2n(bhat), "a": t2n(a)}
    ratios = {
        "float1": 1.0,
        "float07": 0.7,
        "t0d": torch.tensor(1.3),
        "t1d": torch.tensor([0.6, 1.0, 1.7]),
        "t4d": torch.tensor([0.9, 1.2, 2.5]).view(3, 1, 1, 1),
    }
    for mode, spec in (("mono", "P2"), ("rgb", "B2")):
        psf = R.na.create_crosstalk_psf(mode, spec)
        crit = R.lo.PhysicalConsistencyLossSRGB(psf)
        for rk, r in ratios.items():
            bi = bhat.clone().requires_grad_(True)
            loss = crit(bi, a, r)
            loss.backward()
            out[f"{mode}_{rk}_loss"] = t2n(loss)
            out[f"{mode}_{rk}_grad"] = t2n(bi.grad)
            out[f"{mode}_{rk}_align"] = t2n(R.lo.align_exposure_srgb(a, r))
    for rk, r in ratios.items():
        out[f"ratio_{rk}"] = np.asarray(r if not torch.is_tensor(r) else t2n(r), dtype=np.float32)
    # raw-domain PhysicsConsistencyLoss (losses.py:158-192): replicate pad, un-normalised K
    k_mono = R.nl.build_psf_kernels("mono", "P2")
    k_rgb = R.nl.build_psf_kernels("rgb", "B2")
    ratio = torch.tensor([100.0, 250.0, 300.0])
    araw = torch.rand(B, 3, H, W, generator=g) / 200.0
    out["araw"] = t2n(araw)
    out["raw_ratio"] = t2n(ratio)
    for name, k in (("mono", k_mono), ("rgb", k_rgb)):
        for clamp in (True, False):
            crit = R.lo.PhysicsConsistencyLoss(k, device="cpu", clamp_align=clamp)
            bi = bhat.clone().requires_grad_(True)
            loss = crit(bi, araw, ratio)
            loss.backward()
            out[f"raw_{name}_c{int(clamp)}_loss"] = t2n(loss)
            out[f"raw_{name}_c{int(clamp)}_grad"] = t2n(bi.grad)
    save("phys_srgb.npz", **out)


def gen_phys_raw_full(R):
    """PhysicsConsistencyLoss (losses.py:158-192) in its groups == 1 branch: a [Co,1,kh,kw] kernel with Co not in
    {1, C} (expanded along C) and full [Co,C,kh,kw] kernels, with F.l1_loss's channel broadcast against A; plus the
    kernel forms the reference's conv2d rejects (recorded as raising)."""
    import warnings
    g = torch.Generator().manual_seed(21)
    B, H, W = 2, 12, 10
    ratio = torch.tensor([100.0, 250.0])
    cases = {  # name: (C, kernel shape, A channels, clamp_align)
        "c1_co2": (1, (2, 1, 3, 3), 1, True),
        "c3_co4_a1": (3, (4, 1, 3, 3), 1, True),
        "c3_co4_a4": (3, (4, 1, 3, 3), 4, False),
        "full_c3_co2": (3, (2, 3, 3, 3), 2, False),
        "full_c3_co2_a1": (3, (2, 3, 5, 3), 1, True),
        "full_c4_co1_a4": (4, (1, 4, 3, 3), 4, True),
        "full_c3_co3": (3, (3, 3, 3, 3), 3, True),
    }
    out = {"ratio": t2n(ratio), "cases": np.asarray(list(cases))}
    for name, (C, ks, Ca, clamp) in cases.items():
        bhat = torch.rand(B, C, H, W, generator=g)
        k = torch.rand(*ks, generator=g) / (ks[1] * ks[2] * ks[3] / 2)
        a = torch.rand(B, Ca, H, W, generator=g) / 250.0
        out[f"{name}_bhat"], out[f"{name}_k"], out[f"{name}_a"] = t2n(bhat), t2n(k), t2n(a)
        out[f"{name}_clamp"] = np.asarray(int(clamp))
        crit = R.lo.PhysicsConsistencyLoss(k, device="cpu", clamp_align=clamp)
        bi = bhat.clone().requires_grad_(True)
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                loss = crit(bi, a, ratio)
            loss.backward()
        except RuntimeError:
            out[f"{name}_raises"] = np.asarray(1)
            continue
        out[f"{name}_raises"] = np.asarray(0)
        out[f"{name}_loss"] = t2n(loss)
        out[f"{name}_grad"] = t2n(bi.grad)
    save("phys_raw_full.npz", **out)


def gen_ssim_align(R):
    """calculate_ssim's input alignment from the reference's own helpers (metrics/ssim.py:119-167): _to_luma_bt601 and
    _align_pair ('center_crop', 'resize' bilinear / bicubic).  metrics/ssim.py imports torchmetrics at module level
    (absent here): it is loaded with a stub `torchmetrics.image` whose SSIM class is never constructed -- only the two
    helpers run."""
    tm = types.ModuleType("torchmetrics")
    tm.__path__ = []
    tmi = types.ModuleType("torchmetrics.image")
    tmi.StructuralSimilarityIndexMeasure = None
    sys.modules["torchmetrics"], sys.modules["torchmetrics.image"] = tm, tmi
    spec = importlib.util.spec_from_file_location("ref_metrics_ssim", os.path.join(R.ref, "metrics", "ssim.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules["ref_metrics_ssim"] = m  # dataclasses resolve the module by name
    spec.loader.exec_module(m)
    g = torch.Generator().manual_seed(22)
    rgb = torch.rand(2, 3, 29, 33, generator=g)
    out = {"rgb": t2n(rgb), "luma": t2n(m._to_luma_bt601(rgb))}
    tgt = torch.rand(2, 3, 40, 36, generator=g)
    pred = torch.rand(2, 3, 31, 45, generator=g)
    out["tgt"], out["pred"] = t2n(tgt), t2n(pred)
    ct, cp = m._align_pair(tgt, pred, "center_crop")
    out["crop_t"], out["crop_p"] = t2n(ct), t2n(cp)
    for mode in ("bilinear", "bicubic"):
        _, rp = m._align_pair(tgt, pred, "resize", mode)
        out[f"resize_{mode}"] = t2n(rp)
    small = torch.rand(1, 3, 17, 13, generator=g)  # upsampling as well
    out["small"] = t2n(small)
    for mode in ("bilinear", "bicubic"):
        _, rp = m._align_pair(tgt, small, "resize", mode)
        out[f"up_{mode}"] = t2n(rp)
    save("ssim_align.npz", **out)


def gen_phys_cons(R):
    """phys_cons_raw / phys_cons_srgb (metrics/phys_consistency.py:193-368): the variant matrix."""
    import itertools
    import warnings
    g = torch.Generator().manual_seed(13)
    N, C, H, W = 2, 3, 12, 14
    pred = torch.rand(N, C, H, W, generator=g)
    obs = torch.rand(N, C, H, W, generator=g)
    psf3 = torch.rand(C, C, 3, 3, generator=g)
    psf3[torch.arange(C), torch.arange(C), 1, 1] += 2.0  # diagonal-dominant crosstalk
    psf5 = torch.rand(C, C, 5, 5, generator=g) - 0.1  # has negative lobes
    ratios = {
        "scalar": 1.7,
        "batch": torch.tensor([0.8, 1.3]),
        "spatial": torch.rand(N, 1, H, W, generator=g) + 0.5,
        "full": torch.rand(N, C, H, W, generator=g) + 0.5,
    }
    out = {"pred": t2n(pred), "obs": t2n(obs), "psf3": t2n(psf3), "psf5": t2n(psf5)}
    for rk, r in ratios.items():
        out[f"ratio_{rk}"] = np.asarray(r if not torch.is_tensor(r) else t2n(r), dtype=np.float32)
    cases = []
    for fn, padding, crop, robust, rk, psfk, nn_ in itertools.product(
            ("raw", "srgb"), ("reflect", "replicate", "zeros"), ("valid", "same"), ("none", "charbonnier"),
            tuple(ratios), ("psf3", "psf5"), (True, False)):
        if psfk == "psf3" and not nn_:
            continue  # enforce_nonnegative only matters for psf5
        kw = dict(padding=padding, crop=crop, robust=robust, enforce_nonnegative=nn_, return_map=True,
                  reduction="none", eps=1e-3 if robust == "charbonnier" else 1e-12)
        f = R.pc.phys_cons_raw if fn == "raw" else R.pc.phys_cons_srgb
        psf = torch.from_numpy(out[psfk])
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            m, amap = f(pred, obs, psf, ratios[rk], **kw)
        name = f"{fn}|{padding}|{crop}|{robust}|{rk}|{psfk}|{int(nn_)}"
        cases.append(name)
        out["v:" + name] = t2n(m)
        out["m:" + name] = t2n(amap)
    # srgb without clamp, mean/sum reductions, normalize_psf=False
    for red in ("mean", "sum"):
        out[f"srgb_noclamp_{red}"] = t2n(R.pc.phys_cons_srgb(pred, obs, torch.from_numpy(out["psf3"]), 1.4,
                                                              clamp01=False, reduction=red))
        out[f"raw_nonorm_{red}"] = t2n(R.pc.phys_cons_raw(pred, obs, torch.from_numpy(out["psf3"]), 0.9,
                                                           normalize_psf=False, reduction=red))
    save("phys_cons.npz", **out)
    with open(os.path.join(HERE, "phys_cons_cases.json"), "w") as fh:
        json.dump(cases, fh)


def gen_layernorm(R):
    g = torch.Generator().manual_seed(14)
    x = torch.randn(2, 12, 5, 7, generator=g) * 2 + 0.5
    w = torch.randn(12, generator=g) * 0.3 + 1
    b = torch.randn(12, generator=g) * 0.1
    dy = torch.randn(2, 12, 5, 7, generator=g)
    ln = R.au.LayerNorm2d(12)
    with torch.no_grad():
        ln.weight.copy_(w)
        ln.bias.copy_(b)
    xi = x.clone().requires_grad_(True)
    y = ln(xi)
    y.backward(dy)
    save("layernorm.npz", x=t2n(x), w=t2n(w), b=t2n(b), dy=t2n(dy), y=t2n(y), dx=t2n(xi.grad),
         dw=t2n(ln.weight.grad), db=t2n(ln.bias.grad))


def gen_nafblock(R):
    c = 8
    blk = R.arch.NAFBlock(c)
    st = recipe_state([(k, tuple(v.shape)) for k, v in blk.state_dict().items()], seed=15)
    blk.load_state_dict(st)
    g = torch.Generator().manual_seed(16)
    x = torch.randn(2, c, 16, 12, generator=g)
    dy = torch.randn(2, c, 16, 12, generator=g)
    xi = x.clone().requires_grad_(True)
    y = blk(xi)
    y.backward(dy)
    out = {"x": t2n(x), "dy": t2n(dy), "y": t2n(y), "dx": t2n(xi.grad)}
    for k, v in st.items():
        out["p:" + k] = t2n(v)
    for k, p in blk.named_parameters():
        out["g:" + k] = t2n(p.grad)
    save("nafblock.npz", **out)


CFG2 = dict(width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
CFG4 = dict(width=64, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])


def _net_case(R, name, cfg, seed, B, H, W, psf_mode, psf_spec, full=True, ratio=None):
    """NAFNet fwd+bwd under loss = L1(out, gt) + 0.1 * PhysSRGB(out.clamp01, short.clamp01, ratio)."""
    net = R.na.create_newbp_net(in_channels=3, **cfg)
    st = recipe_state([(k, tuple(v.shape)) for k, v in net.state_dict().items()], seed=seed)
    net.load_state_dict(st)
    g = torch.Generator().manual_seed(seed + 1)
    lq = torch.rand(B, 3, H, W, generator=g)
    gt = torch.rand(B, 3, H, W, generator=g)
    r = torch.ones(B, 1, 1, 1) if ratio is None else ratio
    short = (lq * r).clamp(0, 1)
    psf = R.na.create_crosstalk_psf(psf_mode, psf_spec)
    phys = R.lo.PhysicalConsistencyLossSRGB(psf)
    l1 = torch.nn.L1Loss()
    out = net(lq)
    L1 = l1(out, gt)
    Lp = phys(out.clamp(0, 1), short.clamp(0, 1), r)
    loss = L1 + 0.1 * Lp
    loss.backward()
    res = {"lq": t2n(lq), "gt": t2n(gt), "ratio": t2n(r), "out": t2n(out), "L1": t2n(L1), "Phys": t2n(Lp),
           "loss": t2n(loss), "nparams": np.asarray(sum(p.numel() for p in net.parameters()))}
    keys = list(st.keys())
    res["keys"] = np.asarray(keys)
    for k, p in net.named_parameters():
        gr = p.grad
        res["gsum:" + k] = t2n(gr.double().sum())
        res["gnorm:" + k] = t2n(gr.double().norm())
        if full:
            res["g:" + k] = t2n(gr)
    if full:
        for k, v in st.items():
            res["p:" + k] = t2n(v)
    res["seed"] = np.asarray(seed)
    save(name, **res)


def gen_nets(R):
    cfg0 = dict(width=8, enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1])
    _net_case(R, "nafnet_cfg0.npz", cfg0, 100, 2, 32, 32, "rgb", "B2")
    # check_image_size zero padding (NAFNet_arch.py:157-162) + crop (:155): 30x26 is not a multiple of 4
    _net_case(R, "nafnet_cfg0_pad.npz", cfg0, 101, 2, 30, 26, "mono", "P2",
              ratio=torch.tensor([1.0, 1.5]).view(2, 1, 1, 1))
    cfg1 = dict(width=16, enc_blk_nums=[1, 1, 1, 1], middle_blk_num=1, dec_blk_nums=[1, 1, 1, 1])
    _net_case(R, "nafnet_cfg1.npz", cfg1, 102, 2, 64, 64, "mono", "P2", full=False)
    # create_newbp_net defaults (newbp_net_arch.py:31-85): w16, mid 1, no enc/dec; img_channel forced
    net = R.na.create_newbp_net(nafnet_params={"img_channel": 1})
    save("create_defaults.npz", keys=np.asarray(list(net.state_dict().keys())),
         shapes=np.asarray([str(tuple(v.shape)) for v in net.state_dict().values()]))


def gen_cfg_nets(R):
    """BASELINE configs[1] model (w32 [2,2,4,8]/12/[2,2,2,2], rgb B2) at bs 2 x 256^2 and configs[3] model (w64, the
    per-GPU slice at 2 x 64^2): output, loss terms and per-tensor gradient sums / norms (the parameters come from the
    seeded recipe; full tensors would be 117 / 464 MB)."""
    _net_case(R, "nafnet_cfg2.npz", CFG2, 300, 2, 256, 256, "rgb", "B2", full=False)
    _net_case(R, "nafnet_w64.npz", CFG4, 301, 2, 64, 64, "rgb", "B2", full=False)


def _autocast_grads(R, cfg, seed, B, H, W, scale=65536.0):
    """The reference's fp32 and fp16-autocast backward of the _net_case loss (L1 + 0.1 * PhysSRGB) on the same weights
    and batch: per-tensor cosine and relative-norm error of the fp16 gradients against the fp32 ones.  fp16 autocast as
    the reference trains (image_restoration_model.py:255-310: autocast forward + loss, GradScaler-scaled backward,
    unscaled gradients; init scale 2^16), here on the CPU."""
    grads = {}
    for amp in (False, True):
        net = R.na.create_newbp_net(in_channels=3, **cfg)
        st = recipe_state([(k, tuple(v.shape)) for k, v in net.state_dict().items()], seed=seed)
        net.load_state_dict(st)
        g = torch.Generator().manual_seed(seed + 1)
        lq = torch.rand(B, 3, H, W, generator=g)
        gt = torch.rand(B, 3, H, W, generator=g)
        r = torch.ones(B, 1, 1, 1)
        short = (lq * r).clamp(0, 1)
        phys = R.lo.PhysicalConsistencyLossSRGB(R.na.create_crosstalk_psf("rgb", "B2"))
        with torch.autocast("cpu", dtype=torch.float16, enabled=amp):
            out = net(lq)
            loss = F.l1_loss(out, gt) + 0.1 * phys(out.clamp(0, 1), short.clamp(0, 1), r)
        (loss * (scale if amp else 1.0)).backward()
        grads[amp] = {k: p.grad.double() / (scale if amp else 1.0) for k, p in net.named_parameters()}
    keys = list(grads[False].keys())
    cos, rel = [], []
    for k in keys:
        a, b = grads[True][k].flatten(), grads[False][k].flatten()
        nb = b.norm().item()
        cos.append((a @ b).item() / max(a.norm().item() * nb, 1e-300))
        rel.append((a - b).norm().item() / max(nb, 1e-300))
    return np.asarray(keys), np.asarray(cos), np.asarray(rel)


def gen_fp16_grads(R):
    """Calibration of the fp16 headline backward: the reference's OWN fp16-autocast gradients
    against its fp32 gradients, per parameter tensor, at cfg2 (2 x 256^2, the nafnet_cfg2.npz weights and batch) and at
    w64 (2 x 64^2, nafnet_w64.npz)."""
    out = {}
    for tag, cfg, seed, B, H, W in (("cfg2", CFG2, 300, 2, 256, 256), ("w64", CFG4, 301, 2, 64, 64)):
        keys, cos, rel = _autocast_grads(R, cfg, seed, B, H, W)
        out[tag + "_keys"], out[tag + "_cos"], out[tag + "_rel"] = keys, cos, rel
        print(tag, "min cos", cos.min(), "max rel", rel.max(), "median rel", np.median(rel), flush=True)
    save("fp16_grad_calib.npz", **out)


def gen_widths(R):
    """Widths that are not powers of two (the reference accepts any width, NAFNet_arch.py:85-118): w24 / w40 (multiples
    of 8: every precision mode) and w20 (a multiple of 4: the fp32 mode), small U-Nets, full per-tensor gradients."""
    _net_case(R, "nafnet_w24.npz", dict(width=24, enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1]), 400, 2,
              48, 40, "rgb", "B2")
    _net_case(R, "nafnet_w40.npz", dict(width=40, enc_blk_nums=[1, 1, 1], middle_blk_num=2, dec_blk_nums=[1, 1, 1]),
              401, 2, 64, 48, "mono", "P2", full=False)
    _net_case(R, "nafnet_w20.npz", dict(width=20, enc_blk_nums=[1], middle_blk_num=1, dec_blk_nums=[1]), 402, 2, 32, 24,
              "rgb", "B2")


def gen_cfg5(R):
    """BASELINE configs[4]: phys_cons_raw with expo_ratio in {100, 250, 300} at 8 x 3 x 1024^2 (per-GPU slice of bs 32
    over 4 GPUs) + psnr_linear / ssim_linear at data_range 4095 on the unnormalised scale; fp16 inputs too (the metric
    casts to fp32, phys_consistency.py:302-303)."""
    pred, obs, ratios, sl, ss = cfg5_inputs()
    P, O, r = torch.from_numpy(pred), torch.from_numpy(obs), torch.from_numpy(ratios)
    psf = torch.zeros(3, 3, 3, 3)
    k = R.nl.build_psf_kernels("rgb", "B2")
    for c in range(3):
        psf[c, c] = k[c, 0]
    out = {"seed": np.asarray(500), "sum_long": np.asarray(sl), "sum_short": np.asarray(ss), "ratios": ratios,
           "psf": t2n(psf)}
    out["raw_mean"] = t2n(R.pc.phys_cons_raw(P, O, psf, r))
    out["raw_none"] = t2n(R.pc.phys_cons_raw(P, O, psf, r, reduction="none"))
    out["raw_charb_sum"] = t2n(R.pc.phys_cons_raw(P, O, psf, r, reduction="sum", robust="charbonnier",
                                                  padding="replicate", crop="same"))
    out["raw_fp16_none"] = t2n(R.pc.phys_cons_raw(P.half(), O.half(), psf, r, reduction="none"))
    long12 = torch.from_numpy(pred * ratios[:, None, None, None] * np.float32(4095.0))
    short12 = O * 4095.0
    out["psnr4095_none"] = t2n(R.lin.psnr_linear(short12, long12, data_range=4095.0, reduction="none"))
    out["ssim4095_none"] = t2n(R.lin.ssim_linear(short12, long12, data_range=4095.0, reduction="none"))
    save("cfg5_raw.npz", **out)


def gen_train_steps(R):
    """Two full optimize_parameters steps (image_restoration_model.py:247-322, fp32 path :316-320):
    zero_grad -> fwd -> L1 + 0.1*PhysSRGB + 0*sum(p) -> backward -> clip_grad_norm_(0.01) -> AdamW."""
    cfg0 = dict(width=8, enc_blk_nums=[1, 1], middle_blk_num=1, dec_blk_nums=[1, 1])
    net = R.na.create_newbp_net(in_channels=3, **cfg0)
    st = recipe_state([(k, tuple(v.shape)) for k, v in net.state_dict().items()], seed=200)
    net.load_state_dict(st)
    opt = torch.optim.AdamW([{"params": list(net.parameters())}], lr=5e-4, betas=(0.9, 0.999), weight_decay=0.01)
    psf = R.na.create_crosstalk_psf("rgb", "B2")
    phys = R.lo.PhysicalConsistencyLossSRGB(psf)
    l1 = torch.nn.L1Loss()
    res = {}
    g = torch.Generator().manual_seed(201)
    for step in range(2):
        lq = torch.rand(2, 3, 32, 32, generator=g)
        gt = torch.rand(2, 3, 32, 32, generator=g)
        ratio = torch.ones(2, 1, 1, 1)
        short = (lq * ratio).clamp(0, 1)
        opt.zero_grad(set_to_none=True)
        out = net(lq)
        L1 = l1(out, gt)
        Lp = phys(out.clamp(0, 1), short.clamp(0, 1), ratio)
        tot = 0.0 + 1.0 * L1 + 0.1 * Lp
        tot = tot + 0.0 * sum(p.sum() for p in net.parameters())
        tot.backward()
        gn = torch.nn.utils.clip_grad_norm_(net.parameters(), 0.01)
        opt.step()
        res[f"s{step}:lq"] = t2n(lq)
        res[f"s{step}:gt"] = t2n(gt)
        res[f"s{step}:L1"] = t2n(L1)
        res[f"s{step}:Phys"] = t2n(Lp)
        res[f"s{step}:total"] = t2n(tot)
        res[f"s{step}:gradnorm"] = t2n(gn)
        for k, v in net.state_dict().items():
            res[f"s{step}:p:{k}"] = t2n(v)
    for k, v in st.items():
        res["init:" + k] = t2n(v)
    save("train_steps_cfg0.npz", **res)


def gen_color(R):
    with open(os.path.join(R.ref, "standard_tests", "data", "ciede2000_pairs.json")) as fh:
        pairs = json.load(fh)
    lab1 = torch.tensor([[p["L1"], p["a1"], p["b1"]] for p in pairs], dtype=torch.float32).T.reshape(1, 3, 1, -1)
    lab2 = torch.tensor([[p["L2"], p["a2"], p["b2"]] for p in pairs], dtype=torch.float32).T.reshape(1, 3, 1, -1)
    gold = np.asarray([p["de00"] for p in pairs], dtype=np.float32)
    g = torch.Generator().manual_seed(17)
    rl1 = torch.stack([torch.rand(2, 9, 11, generator=g) * 100, torch.randn(2, 9, 11, generator=g) * 40,
                       torch.randn(2, 9, 11, generator=g) * 40], 1)
    rl2 = rl1 + torch.randn(rl1.shape, generator=g) * 5
    loss_sharma = R.lo.DeltaE00Loss._ciede2000(lab1, lab2, 1e-6)
    loss_rand = R.lo.DeltaE00Loss._ciede2000(rl1, rl2, 1e-6)
    met_sharma = R.ce._deltaE00_lab_map(lab1, lab2, kL=1.0, kC=1.0, kH=1.0, eps=1e-12)
    met_rand = R.ce._deltaE00_lab_map(rl1, rl2, kL=1.0, kC=1.0, kH=1.0, eps=1e-12)
    # gradient of the loss-form ΔE00 w.r.t. Lab1 (for the on-device backward)
    li = rl1.clone().requires_grad_(True)
    R.lo.DeltaE00Loss._ciede2000(li, rl2, 1e-6).mean().backward()
    save("ciede2000.npz", lab1=t2n(lab1), lab2=t2n(lab2), sharma_gold=gold, loss_sharma=t2n(loss_sharma),
         rl1=t2n(rl1), rl2=t2n(rl2), loss_rand=t2n(loss_rand), met_sharma=t2n(met_sharma),
         met_rand=t2n(met_rand), loss_rand_grad=t2n(li.grad))


def gen_linear(R):
    g = torch.Generator().manual_seed(18)
    a = torch.rand(3, 3, 40, 36, generator=g)
    b = (a + 0.05 * torch.randn(a.shape, generator=g)).clamp(0, 1)
    out = {"a": t2n(a), "b": t2n(b)}
    out["psnr_none"] = t2n(R.lin.psnr_linear(b, a, reduction="none"))
    out["psnr_mean"] = t2n(R.lin.psnr_linear(b, a))
    out["psnr_4095"] = t2n(R.lin.psnr_linear(b * 4095, a * 4095, data_range=4095.0, reduction="none"))
    out["ssim_none"] = t2n(R.lin.ssim_linear(b, a, reduction="none"))
    out["ssim_mean"] = t2n(R.lin.ssim_linear(b, a))
    out["ssim_chan"] = t2n(R.lin.ssim_linear(b, a, reduction="none", channel_aggregate="none"))
    out["calc_psnr"] = np.asarray(R.psnr.calculate_psnr(a, b, data_range=1.0))
    save("linear_metrics.npz", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated generator names (default: all)")
    args = ap.parse_args()
    torch.set_num_threads(8)
    R = load_reference(args.ref)
    R.ref = args.ref
    gens = dict(psf=gen_psf, phys_srgb=gen_phys_srgb, phys_raw_full=gen_phys_raw_full, phys_cons=gen_phys_cons, layernorm=gen_layernorm,
                nafblock=gen_nafblock, nets=gen_nets, cfg_nets=gen_cfg_nets, widths=gen_widths, cfg5=gen_cfg5,
                train_steps=gen_train_steps, color=gen_color, linear=gen_linear,
                ssim_align=gen_ssim_align, fp16_grads=gen_fp16_grads)
    for name, fn in gens.items():
        if not args.only or name in args.only.split(","):
            fn(R)


if __name__ == "__main__":
    main()
