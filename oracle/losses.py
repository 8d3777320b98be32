"""Oracle: HybridLoss terms (pixel, SSIM, ΔE00) and the linear-domain metrics.

Test infrastructure only (see oracle/__init__.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def l1(a, b):
    """nn.L1Loss (losses.py:249,332): mean |a-b|."""
    return (a - b).abs().mean()


def charbonnier(a, b, eps=1e-12):
    """charbonnier_loss (NAFNet_base/basicsr/models/losses/losses.py:29-31): sqrt(d^2 + eps), eps NOT squared."""
    d = a - b
    return torch.sqrt(d * d + eps).mean()


# ---- kornia==0.6.12 SSIMLoss, restated (requirements.txt:25; call site losses.py:146-155) -------------
def gaussian1d(ks=11, sigma=1.5, dtype=torch.float32):
    """kornia.filters.kernels.gaussian: x = arange(ks) - ks//2, exp(-x^2/(2 s^2)), normalised."""
    x = torch.arange(ks, dtype=dtype) - ks // 2
    g = torch.exp(-x.pow(2.0) / (2 * sigma ** 2))
    return g / g.sum()


def _filter2d_reflect(x, k1d):
    """kornia filter2d(border_type='reflect', padding='same') with the 2-D outer-product window."""
    ks = k1d.numel()
    k2 = torch.matmul(k1d.unsqueeze(-1), k1d.unsqueeze(-1).t())
    C = x.shape[1]
    p = ks // 2
    xp = F.pad(x, (p, p, p, p), mode="reflect")
    return F.conv2d(xp, k2.expand(C, 1, ks, ks).to(x.dtype).to(x.device), groups=C)


def ssim_map(img1, img2, window_size=11, max_val=1.0, eps=1e-12):
    """kornia.metrics.ssim (0.6.12): C1=(0.01L)^2, C2=(0.03L)^2, num/(den+eps)."""
    k = gaussian1d(window_size, 1.5).to(img1.device)
    C1 = (0.01 * max_val) ** 2
    C2 = (0.03 * max_val) ** 2
    mu1 = _filter2d_reflect(img1, k)
    mu2 = _filter2d_reflect(img2, k)
    mu1_sq, mu2_sq, mu12 = mu1 ** 2, mu2 ** 2, mu1 * mu2
    s1 = _filter2d_reflect(img1 ** 2, k) - mu1_sq
    s2 = _filter2d_reflect(img2 ** 2, k) - mu2_sq
    s12 = _filter2d_reflect(img1 * img2, k) - mu12
    num = (2.0 * mu12 + C1) * (2.0 * s12 + C2)
    den = (mu1_sq + mu2_sq + C1) * (s1 + s2 + C2)
    return num / (den + eps)


def ssim_loss(gen01, tgt01, window_size=11, max_val=1.0):
    """SSIMLoss.forward (losses.py:154-155) -> kornia ssim_loss: mean(clamp((1-ssim)/2, 0, 1))."""
    m = ssim_map(gen01.clamp(0, 1), tgt01.clamp(0, 1), window_size, max_val)
    return torch.clamp((1.0 - m) / 2, min=0, max=1).mean()


# ---- kornia==0.6.12 rgb_to_lab, restated (call site losses.py:140-141) --------------------------------
def rgb_to_lab(image):
    """sRGB linearise (0.04045 / 12.92 / 2.4) -> XYZ (D65) -> Lab (threshold 0.008856, 7.787t + 4/29)."""
    lin = torch.where(image > 0.04045, torch.pow((image + 0.055) / 1.055, 2.4), image / 12.92)
    r, g, b = lin[:, 0], lin[:, 1], lin[:, 2]
    x = 0.412453 * r + 0.357580 * g + 0.180423 * b
    y = 0.212671 * r + 0.715160 * g + 0.072169 * b
    z = 0.019334 * r + 0.119193 * g + 0.950227 * b
    xyz = torch.stack([x, y, z], 1)
    white = torch.tensor([0.95047, 1.0, 1.08883], dtype=xyz.dtype).view(1, 3, 1, 1)
    xyz_n = xyz / white
    thr = 0.008856
    power = torch.pow(xyz_n.clamp(min=thr), 1 / 3.0)
    scale = 7.787 * xyz_n + 4.0 / 29.0
    f = torch.where(xyz_n > thr, power, scale)
    fx, fy, fz = f[:, 0], f[:, 1], f[:, 2]
    L = (116.0 * fy) - 16.0
    a = 500.0 * (fx - fy)
    bb = 200.0 * (fy - fz)
    return torch.stack([L, a, bb], 1)


def ciede2000_loss_form(Lab1, Lab2, eps=1e-6):
    """DeltaE00Loss._ciede2000 (losses.py:98-136) — the non-standard loss formula, restated term by term."""
    L1, a1, b1 = Lab1[:, 0], Lab1[:, 1], Lab1[:, 2]
    L2, a2, b2 = Lab2[:, 0], Lab2[:, 1], Lab2[:, 2]
    pi = torch.pi
    C1 = torch.sqrt(a1 * a1 + b1 * b1 + eps)
    C2 = torch.sqrt(a2 * a2 + b2 * b2 + eps)
    Cb = 0.5 * (C1 + C2)
    G = 0.5 * (1 - torch.sqrt((Cb ** 7) / ((Cb ** 7) + (25 ** 7) + eps)))
    a1p, a2p = (1 + G) * a1, (1 + G) * a2
    C1p = torch.sqrt(a1p * a1p + b1 * b1 + eps)
    C2p = torch.sqrt(a2p * a2p + b2 * b2 + eps)
    h1p = torch.atan2(b1, a1p) % (2 * pi)
    h2p = torch.atan2(b2, a2p) % (2 * pi)
    dLp = L2 - L1
    dCp = C2p - C1p
    dhp = h2p - h1p
    dhp = dhp - (2 * pi) * (dhp > pi) + (2 * pi) * (dhp < -pi)
    dHp = 2 * torch.sqrt(C1p * C2p + eps) * torch.sin(dhp / 2)
    Lb = 0.5 * (L1 + L2)
    Cbp = 0.5 * (C1p + C2p)
    hs = h1p + h2p
    hbp = hs / 2 - pi * (torch.abs(h1p - h2p) > pi) + (2 * pi) * (hs < 0)
    d30, d6, d63 = (torch.deg2rad(torch.tensor(v)) for v in (30.0, 6.0, 63.0))
    T = (1 - 0.17 * torch.cos(hbp - d30) + 0.24 * torch.cos(2 * hbp) + 0.32 * torch.cos(3 * hbp + d6)
         - 0.20 * torch.cos(4 * hbp - d63))
    dro = 30 * torch.exp(-((torch.rad2deg(hbp) - 275) / 25) ** 2)
    RC = 2 * torch.sqrt((Cbp ** 7) / ((Cbp ** 7) + (25 ** 7) + eps))
    SL = 1 + (0.015 * ((Lb - 50) ** 2)) / torch.sqrt(20 + (Lb - 50) ** 2 + eps)
    SC = 1 + 0.045 * Cbp
    SH = 1 + 0.015 * Cbp * T
    RT = -torch.sin(torch.deg2rad(dro)) * RC
    return torch.sqrt((dLp / SL) ** 2 + (dCp / SC) ** 2 + (dHp / SH) ** 2 + RT * (dCp / SC) * (dHp / SH) + eps)


def deltae00_loss(gen01, tgt01, eps=1e-6):
    """DeltaE00Loss.forward (losses.py:138-143)."""
    return ciede2000_loss_form(rgb_to_lab(gen01.clamp(0, 1)), rgb_to_lab(tgt01.clamp(0, 1)), eps).mean()


def deltae00_metric_map(lab1, lab2, kL=1.0, kC=1.0, kH=1.0, eps=1e-12):
    """_deltaE00_lab_map (metrics/color_error.py:105-210): the metric-form ΔE00 (differs from the loss form):
    hue angles NOT wrapped, c1'c2'==0 special cases, R_T = -sin(2Δθ)R_C, /(k·S+eps), sqrt(clamp>=0)."""
    pi = torch.pi
    L1, a1, b1 = lab1[:, 0], lab1[:, 1], lab1[:, 2]
    L2, a2, b2 = lab2[:, 0], lab2[:, 1], lab2[:, 2]
    c1 = torch.sqrt(a1 * a1 + b1 * b1 + eps)
    c2 = torch.sqrt(a2 * a2 + b2 * b2 + eps)
    cb7 = (0.5 * (c1 + c2)).pow(7)
    p25 = torch.tensor(25.0 ** 7, dtype=lab1.dtype)
    g = 0.5 * (1.0 - torch.sqrt(cb7 / (cb7 + p25 + eps)))
    a1p, a2p = (1.0 + g) * a1, (1.0 + g) * a2
    c1p = torch.sqrt(a1p * a1p + b1 * b1 + eps)
    c2p = torch.sqrt(a2p * a2p + b2 * b2 + eps)
    h1p = torch.atan2(b1, a1p)
    h2p = torch.atan2(b2, a2p)
    dLp = L2 - L1
    dCp = c2p - c1p
    valid = (c1p * c2p) != 0.0
    diff = h2p - h1p
    dh = torch.zeros_like(h1p)
    dh = torch.where(valid & (torch.abs(diff) <= pi), diff, dh)
    dh = torch.where(valid & (diff > pi), diff - 2.0 * pi, dh)
    dh = torch.where(valid & (diff < -pi), diff + 2.0 * pi, dh)
    dHp = 2.0 * torch.sqrt(c1p * c2p + eps) * torch.sin(dh / 2.0)
    Lbp = 0.5 * (L1 + L2)
    Cbp = 0.5 * (c1p + c2p)
    hs = h1p + h2p
    ad = torch.abs(h1p - h2p)
    hb = torch.where(~valid, hs, torch.where(ad <= pi, 0.5 * hs,
                     torch.where(hs < 2.0 * pi, 0.5 * (hs + 2.0 * pi), 0.5 * (hs - 2.0 * pi))))
    rad = lambda d: float(d) * pi / 180.0  # noqa: E731
    T = (1.0 - 0.17 * torch.cos(hb - rad(30.0)) + 0.24 * torch.cos(2.0 * hb) + 0.32 * torch.cos(3.0 * hb + rad(6.0))
         - 0.20 * torch.cos(4.0 * hb - rad(63.0)))
    dtheta = rad(30.0) * torch.exp(-(((hb * 180.0 / pi) - 275.0) / 25.0) ** 2)
    RC = 2.0 * torch.sqrt((Cbp.pow(7)) / (Cbp.pow(7) + p25 + eps))
    RT = -torch.sin(2.0 * dtheta) * RC
    SL = 1.0 + (0.015 * (Lbp - 50.0) ** 2) / torch.sqrt(20.0 + (Lbp - 50.0) ** 2 + eps)
    SC = 1.0 + 0.045 * Cbp
    SH = 1.0 + 0.015 * Cbp * T
    tL = dLp / (kL * SL + eps)
    tC = dCp / (kC * SC + eps)
    tH = dHp / (kH * SH + eps)
    return torch.sqrt(torch.clamp(tL * tL + tC * tC + tH * tH + RT * tC * tH, min=0.0))


# ---- metrics/linear.py and metrics/psnr.py restated ---------------------------------------------------
def psnr_linear(pred, target, data_range=1.0, reduction="mean", eps=1e-12):
    """psnr_linear (metrics/linear.py:140-215): per-sample float64 MSE, inf when mse <= eps."""
    if pred.ndim == 3:
        pred, target = pred[None], target[None]
    mse = (pred - target).to(torch.float64).pow(2).flatten(1).mean(dim=1)
    p = 10.0 * torch.log10((float(data_range) ** 2) / torch.maximum(mse, torch.full_like(mse, eps)))
    p = torch.where(mse <= eps, torch.full_like(p, float("inf")), p)
    return {"mean": p.mean(0), "sum": p.sum(0), "none": p}[reduction]


def calculate_psnr(img_true, img_pred, data_range):
    """calculate_psnr (metrics/psnr.py:18-67)."""
    mse = torch.mean((img_true.double() - img_pred.double()) ** 2)
    if torch.isclose(mse, mse.new_tensor(0.0), atol=1e-12):
        return float("inf")
    return float(10.0 * torch.log10((data_range ** 2) / mse))


def ssim_linear(pred, target, data_range=1.0, kernel_size=11, sigma=1.5, k1=0.01, k2=0.03,
                reduction="mean", channel_aggregate="mean", eps=1e-12):
    """ssim_linear (metrics/linear.py:218-324): float64-built window, reflect pad, variance clamp >= 0."""
    if pred.ndim == 3:
        pred, target = pred[None], target[None]
    n, c, h, w = pred.shape
    coords = torch.arange(kernel_size, dtype=torch.float64) - (kernel_size - 1) / 2.0
    k1d = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    k2d = k1d[:, None] * k1d[None, :]
    k2d = (k2d.to(pred.dtype) / k2d.to(pred.dtype).sum()).view(1, 1, kernel_size, kernel_size).repeat(c, 1, 1, 1)
    p = kernel_size // 2
    xp = F.pad(pred, (p, p, p, p), mode="reflect")
    yp = F.pad(target, (p, p, p, p), mode="reflect")
    mx = F.conv2d(xp, k2d, groups=c)
    my = F.conv2d(yp, k2d, groups=c)
    sx = torch.clamp(F.conv2d(xp * xp, k2d, groups=c) - mx.pow(2), min=0.0)
    sy = torch.clamp(F.conv2d(yp * yp, k2d, groups=c) - my.pow(2), min=0.0)
    sxy = F.conv2d(xp * yp, k2d, groups=c) - mx * my
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    m = (2 * mx * my + c1) * (2 * sxy + c2) / ((mx.pow(2) + my.pow(2) + c1) * (sx + sy + c2) + eps)
    pc = m.flatten(2).mean(dim=2)
    pi = pc.mean(dim=1) if channel_aggregate == "mean" else pc
    return {"mean": pi.mean(0), "sum": pi.sum(0), "none": pi}[reduction]


def luma_bt601(images):
    """metrics/ssim.py:119-131 (_to_luma_bt601)."""
    return 0.2989 * images[:, 0:1] + 0.5870 * images[:, 1:2] + 0.1140 * images[:, 2:3]


def ssim_align_pair(target, prediction, policy, mode="bilinear"):
    """metrics/ssim.py:134-167 (_align_pair): resize the prediction to the target's size, or centre-crop both."""
    if policy is None:
        return target, prediction
    if policy == "resize":
        return target, F.interpolate(prediction, size=target.shape[-2:], mode=mode, align_corners=False)
    h, w = min(target.shape[-2], prediction.shape[-2]), min(target.shape[-1], prediction.shape[-1])

    def crop(x):
        top, left = max((x.shape[-2] - h) // 2, 0), max((x.shape[-1] - w) // 2, 0)
        return x[:, :, top:top + h, left:left + w]

    return crop(target), crop(prediction)


# ---- torchvision==0.17.1 vgg19 / vgg16 `features` and lpips==0.1.4, restated (losses.py:32-69, 265-274) ----
# Weights: torchvision's pretrained files are a download (unavailable offline), so the oracle takes the state_dict
# the caller passes (the product's deterministic synthetic one in the tests) -- parity unpinned for real weights.
VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


def vgg_features(sd, x, cfg=VGG19_CFG, n_modules=36, taps=()):
    """torchvision vgg.features[:n_modules] (conv 3x3 pad 1 -> ReLU, 2x2 max pool); returns (out, {relu idx: map})."""
    h, idx, res = x, 0, {}
    for v in cfg:
        if idx >= n_modules:
            break
        if v == "M":
            h = F.max_pool2d(h, 2)
            idx += 1
        else:
            h = F.relu(F.conv2d(h, sd[f"{idx}.weight"].to(x.dtype), sd[f"{idx}.bias"].to(x.dtype), padding=1))
            if idx + 1 in taps:
                res[idx + 1] = h
            idx += 2
    return h, res


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def perceptual_loss(sd, gen, tgt):
    """PerceptualLoss.forward (losses.py:54-69): clamp01 -> ImageNet normalisation -> features[:36] -> MSE."""
    mean = torch.tensor(IMAGENET_MEAN, dtype=gen.dtype).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=gen.dtype).view(1, 3, 1, 1)
    fg, _ = vgg_features(sd, (gen.clamp(0, 1) - mean) / std)
    ft, _ = vgg_features(sd, (tgt.clamp(0, 1) - mean) / std)
    return F.mse_loss(fg, ft)


LPIPS_SHIFT = (-0.030, -0.088, -0.188)
LPIPS_SCALE = (0.458, 0.448, 0.450)
LPIPS_VGG_TAPS = (3, 8, 15, 22, 29)


def lpips_vgg(feats, lins, in0, in1):
    """lpips.LPIPS(net='vgg').forward(in0, in1) per image [N,1,1,1] (inputs taken as [-1,1], no normalize): ScalingLayer,
    VGG16 relu1_2..relu5_3 taps, channel unit-normalisation (eps 1e-10), squared difference, lin head, spatial mean."""
    shift = torch.tensor(LPIPS_SHIFT, dtype=in0.dtype).view(1, 3, 1, 1)
    scale = torch.tensor(LPIPS_SCALE, dtype=in0.dtype).view(1, 3, 1, 1)
    _, t0 = vgg_features(feats, (in0 - shift) / scale, VGG16_CFG, 30, LPIPS_VGG_TAPS)
    _, t1 = vgg_features(feats, (in1 - shift) / scale, VGG16_CFG, 30, LPIPS_VGG_TAPS)
    val = 0
    for k, tap in enumerate(LPIPS_VGG_TAPS):
        u = t0[tap] / (t0[tap].pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
        v = t1[tap] / (t1[tap].pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
        d = ((u - v) ** 2 * lins[k].to(in0.dtype).view(1, -1, 1, 1)).sum(1, keepdim=True)
        val = val + d.mean((2, 3), keepdim=True)
    return val


# torchvision alexnet.features (lpips net='alex' slices: relu1 | pool, conv, relu2 | pool, conv, relu3 | conv, relu4 |
# conv, relu5): (module index, stride, pad) of each conv
ALEX_CONVS = ((0, 4, 2), (3, 1, 2), (6, 1, 1), (8, 1, 1), (10, 1, 1))


def lpips_alex(feats, lins, in0, in1):
    """lpips.LPIPS(net='alex').forward(in0, in1) per image [N,1,1,1] (lpips 0.1.4 pretrained_networks.alexnet +
    the same head as lpips_vgg)."""
    shift = torch.tensor(LPIPS_SHIFT, dtype=in0.dtype).view(1, 3, 1, 1)
    scale = torch.tensor(LPIPS_SCALE, dtype=in0.dtype).view(1, 3, 1, 1)

    def taps(x):
        h, out = (x - shift) / scale, []
        for i, (idx, st, pad) in enumerate(ALEX_CONVS):
            if i in (1, 2):
                h = F.max_pool2d(h, 3, 2)
            h = F.relu(F.conv2d(h, feats[f"{idx}.weight"].to(x.dtype), feats[f"{idx}.bias"].to(x.dtype), stride=st,
                                padding=pad))
            out.append(h)
        return out

    t0, t1 = taps(in0), taps(in1)
    val = 0
    for k in range(5):
        u = t0[k] / (t0[k].pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
        v = t1[k] / (t1[k].pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
        val = val + ((u - v) ** 2 * lins[k].to(in0.dtype).view(1, -1, 1, 1)).sum(1, keepdim=True).mean((2, 3),
                                                                                                     keepdim=True)
    return val


_ = math  # keep import for callers that use math constants
