"""Oracle: one training step (ImageRestorationModel.optimize_parameters, fp32 path) on CPU.

Test infrastructure only (see oracle/__init__.py).  Also the `cpu_baseline` leg
of bench.py (`kind: "port"`).
"""
from __future__ import annotations

from typing import Dict

import torch

from . import losses as L
from . import nafnet as N
from . import physics as P


class OracleTrainer:
    """image_restoration_model.py:247-322 (fp32 branch :316-320) with HybridLossPlus term order
    (NewBP_model/losses.py:318-372).  The VGG19 perceptual and LPIPS(vgg) terms take the caller's weights
    (`vgg19_sd`, `lpips_parts` = (vgg16 features sd, [5 lin weights])): pretrained ones are unavailable offline."""

    def __init__(self, params: Dict[str, torch.Tensor], cfg: dict, psf_mode="rgb", psf_spec="B2",
                 w_l1=1.0, w_ssim=0.0, w_phys=0.1, w_de=0.0, lr=5e-4, betas=(0.9, 0.999), wd=0.01, eps=1e-8,
                 max_norm=0.01, w_perc=0.0, w_lpips=0.0, vgg19_sd=None, lpips_parts=None):
        self.P = {k: v.detach().clone().float().requires_grad_(True) for k, v in params.items()}
        self.cfg = cfg
        self.k = P.normalize_psf(P.build_psf_kernels(psf_mode, psf_spec))
        self.w = dict(l1=w_l1, ssim=w_ssim, phys=w_phys, de=w_de, perc=w_perc, lpips=w_lpips)
        self.vgg19_sd, self.lpips_parts = vgg19_sd, lpips_parts
        self.lr, self.betas, self.wd, self.eps, self.max_norm = lr, betas, wd, eps, max_norm
        self.m = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.t = 0

    def loss(self, lq, gt, short, ratio):
        out = N.nafnet(self.P, lq, **self.cfg)
        logs = {}
        tot = 0.0
        l1 = L.l1(out, gt)
        logs["L1_raw"] = l1.detach()
        tot = tot + self.w["l1"] * l1
        o01, g01 = out.clamp(0, 1), gt.clamp(0, 1)
        if self.w["perc"]:
            pe = L.perceptual_loss(self.vgg19_sd, o01, g01)
            logs["Perc"] = pe.detach()
            tot = tot + self.w["perc"] * pe
        if self.w["lpips"]:
            lp = L.lpips_vgg(*self.lpips_parts, o01, g01).mean()
            logs["LPIPS"] = lp.detach()
            tot = tot + self.w["lpips"] * lp
        if self.w["de"]:
            de = L.deltae00_loss(o01, g01)
            logs["DeltaE"] = de.detach()
            tot = tot + self.w["de"] * de
        if self.w["ssim"]:
            ss = L.ssim_loss(o01, g01)
            logs["SSIM"] = ss.detach()
            tot = tot + self.w["ssim"] * ss
        if self.w["phys"]:
            ph = P.phys_srgb_loss(o01, short.clamp(0, 1), ratio, self.k)
            logs["Phys"] = ph.detach()
            tot = tot + self.w["phys"] * ph
        tot = tot + 0.0 * sum(p.sum() for p in self.P.values())  # image_restoration_model.py:306
        logs["Total"] = tot.detach()
        return out, tot, logs

    @torch.no_grad()
    def _clip_adamw(self):
        # clip_grad_norm_ (max_norm 0.01, :319): coef = max_norm / (norm + 1e-6), clamped to 1
        norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in self.P.values())).float()
        coef = torch.clamp(self.max_norm / (norm + 1e-6), max=1.0)
        self.t += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        for k, p in self.P.items():
            g = p.grad * coef
            p.mul_(1 - self.lr * self.wd)  # torch.optim.AdamW decoupled decay
            self.m[k].lerp_(g, 1 - b1)
            self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (self.v[k].sqrt() / (bc2 ** 0.5)).add_(self.eps)
            p.addcdiv_(self.m[k], denom, value=-self.lr / bc1)
        return norm

    def step(self, lq, gt, short, ratio):
        for p in self.P.values():
            p.grad = None
        out, tot, logs = self.loss(lq, gt, short, ratio)
        tot.backward()
        logs["gradnorm"] = self._clip_adamw()
        return out, logs
