"""metrics.phys_consistency on MI355X (reference: metrics/phys_consistency.py).

phys_cons_raw / phys_cons_srgb: no-grad physics-consistency metrics with the reference's argument names,
defaults, validation errors (TypeError / ValueError / RuntimeWarning) and outputs.  The PSF application, exposure
scaling, clamp, crop, robust penalty and per-sample reduction are one HIP kernel (nbp_phys_cons); the PSF
preparation (<= a few hundred floats) happens on the host like the reference's tiny tensor ops.
"""
from __future__ import annotations

import warnings
from typing import Literal, Tuple

import torch
from torch import Tensor

from .. import _lib
from .._lib import call, query

__all__ = ["phys_cons_raw", "phys_cons_srgb"]

_PAD = {"zeros": 0, "replicate": 1, "reflect": 2}


def _ensure_nchw(pred: Tensor, obs: Tensor) -> Tuple[Tensor, Tensor]:
    """phys_consistency.py:37-62."""
    if not isinstance(pred, Tensor) or not isinstance(obs, Tensor):
        raise TypeError("phys_consistency metrics expect torch.Tensor inputs.")
    if pred.shape != obs.shape:
        raise ValueError(f"`pred` and `obs` must share identical shape, got {tuple(pred.shape)} vs {tuple(obs.shape)}.")
    if pred.device != obs.device:
        raise ValueError("`pred` and `obs` must reside on the same device.")
    if pred.ndim == 3:
        pred, obs = pred.unsqueeze(0), obs.unsqueeze(0)
    elif pred.ndim != 4:
        raise ValueError("Inputs must have 3 (C,H,W) or 4 (N,C,H,W) dimensions; "
                         f"received tensor with shape {tuple(pred.shape)}.")
    if pred.shape[1] == 0:
        raise ValueError("Channel dimension must be positive.")
    pred = pred.detach().to(torch.float32).contiguous()
    obs = obs.detach().to(torch.float32).contiguous()
    _lib.require_cuda(pred, obs)
    flag = torch.zeros(2, dtype=torch.int32, device=pred.device)
    call("all_finite", pred, pred.numel(), flag[0:1])
    call("all_finite", obs, obs.numel(), flag[1:2])
    f = flag.cpu()
    if int(f[0]):
        raise ValueError("`pred` contains NaN or Inf values.")
    if int(f[1]):
        raise ValueError("`obs` contains NaN or Inf values.")
    return pred, obs


def _prepare_psf(psf, *, in_channels, out_channels, normalize, enforce_nonnegative, eps) -> Tensor:
    """phys_consistency.py:75-127 (host side; the normalisation is per output channel)."""
    if not isinstance(psf, Tensor):
        raise TypeError("`psf` must be a torch.Tensor.")
    if psf.ndim == 2:
        psf = psf.unsqueeze(0).unsqueeze(0)
    if psf.ndim != 4:
        raise ValueError(f"`psf` must have shape [C_out, C_in, kh, kw]; received tensor with shape {tuple(psf.shape)}.")
    c_out, c_in, kh, kw = psf.shape
    if c_out != out_channels:
        raise ValueError(f"PSF output channels ({c_out}) must match observation channels ({out_channels}).")
    if c_in != in_channels:
        raise ValueError(f"PSF input channels ({c_in}) must match prediction channels ({in_channels}).")
    if kh < 1 or kw < 1:
        raise ValueError("PSF kernel height/width must be >= 1.")
    if kh % 2 == 0 or kw % 2 == 0:
        raise ValueError("PSF kernels must have odd spatial dimensions to avoid half-pixel shifts. "
                         "Please supply odd-sized kernels (e.g., 3/5/7).")
    p = psf.detach().to("cpu", torch.float32)
    if enforce_nonnegative:
        p = p.clamp_min(0)
    if normalize:
        sums = p.view(c_out, -1).sum(dim=1)
        zero = sums.abs() < eps
        if zero.any():
            warnings.warn("PSF channel sums near zero detected during normalisation; clamping to preserve stability.",
                          RuntimeWarning)
        p = p / torch.where(zero, torch.ones_like(sums), sums).view(c_out, 1, 1, 1)
    return p


def _ratio(expo_ratio, ref: Tensor, C: int):
    """_expand_exposure (phys_consistency.py:160-190) -> (array, mode 0 [N] / 1 [N,1,H,W] / 2 [N,C,H,W])."""
    N, _, H, W = ref.shape
    if torch.is_tensor(expo_ratio):
        r = expo_ratio.to(device=ref.device, dtype=torch.float32)
    else:
        r = torch.tensor(float(expo_ratio), device=ref.device, dtype=torch.float32)
    if r.ndim == 0:
        return r.view(1).expand(N).contiguous(), 0
    if r.ndim == 1:
        if r.shape[0] != N:
            raise ValueError(f"Exposure ratio length ({r.shape[0]}) must match batch size ({N}).")
        return r.contiguous(), 0
    if r.ndim == 4:
        if r.shape[0] != N:
            raise ValueError(f"Exposure ratio batch dimension ({r.shape[0]}) must match batch size ({N}).")
        if r.shape[1] not in (1, C):
            raise ValueError(f"Exposure ratio channel dimension ({r.shape[1]}) incompatible with data channels ({C}).")
        if r.shape[1] == 1:
            return r.expand(N, 1, H, W).contiguous(), 1
        return r.expand(N, C, H, W).contiguous(), 2
    raise ValueError("Exposure ratio must be scalar, [N], or [N,1,H,W]/[N,C,H,W] for broadcasting.")


def _core(pred, obs, *, psf, expo_ratio, reduction, padding, normalize_psf, enforce_nonnegative, crop, robust,
          return_map, clamp01, eps):
    """_phys_cons_core (phys_consistency.py:193-255)."""
    if eps <= 0:
        raise ValueError(f"`eps` must be positive, received {eps}.")
    if robust not in {"none", "charbonnier"}:
        raise ValueError(f"Unsupported robust loss '{robust}'.")
    if crop not in {"valid", "same"}:
        raise ValueError(f"Unsupported crop mode '{crop}'.")
    if padding not in _PAD:
        raise ValueError(f"Unsupported padding mode '{padding}'.")
    if reduction not in {"mean", "sum", "none"}:
        raise ValueError(f"Unsupported reduction '{reduction}'. Choose from 'mean', 'sum', 'none'.")
    N, Ci, H, W = pred.shape
    Co = obs.shape[1]
    k = _prepare_psf(psf, in_channels=Ci, out_channels=Co, normalize=normalize_psf,
                     enforce_nonnegative=enforce_nonnegative, eps=eps)
    kh, kw = k.shape[-2:]
    kd = k.to(pred.device).contiguous()
    r, rmode = _ratio(expo_ratio, pred, Co)
    valid = crop == "valid"
    Ho, Wo = (H - 2 * (kh // 2), W - 2 * (kw // 2)) if valid else (H, W)
    amap = torch.empty(N, Co, Ho, Wo, device=pred.device) if return_map else None
    ws = torch.empty(query("phys_cons_workspace_doubles", N, H, W), dtype=torch.float64, device=pred.device)
    out = torch.empty(N + 2, device=pred.device)
    call("phys_cons", pred, obs, kd, r, rmode, N, Ci, Co, H, W, kh, kw, _PAD[padding], int(valid), int(clamp01),
         int(robust == "charbonnier"), float(eps), amap, ws, out)
    metric = {"none": out[:N], "mean": out[N], "sum": out[N + 1]}[reduction]
    return (metric, amap) if return_map else metric


@torch.no_grad()
def phys_cons_raw(pred_linear: Tensor, obs_short_linear: Tensor, psf: Tensor, expo_ratio, *,
                  reduction: Literal["mean", "sum", "none"] = "mean", padding="reflect", normalize_psf: bool = True,
                  enforce_nonnegative: bool = False, crop="valid", robust="none", return_map: bool = False,
                  eps: float = 1e-12):
    """phys_consistency.py:260-319."""
    pred, obs = _ensure_nchw(pred_linear, obs_short_linear)
    return _core(pred, obs, psf=psf, expo_ratio=expo_ratio, reduction=reduction, padding=padding,
                 normalize_psf=normalize_psf, enforce_nonnegative=enforce_nonnegative, crop=crop, robust=robust,
                 return_map=return_map, clamp01=False, eps=eps)


@torch.no_grad()
def phys_cons_srgb(pred_srgb: Tensor, obs_short_srgb: Tensor, psf: Tensor, expo_ratio=1.0, *,
                   reduction: Literal["mean", "sum", "none"] = "mean", padding="reflect", normalize_psf: bool = True,
                   enforce_nonnegative: bool = False, crop="valid", robust="none", clamp01: bool = True,
                   return_map: bool = False, eps: float = 1e-12):
    """phys_consistency.py:323-368."""
    pred, obs = _ensure_nchw(pred_srgb, obs_short_srgb)
    return _core(pred, obs, psf=psf, expo_ratio=expo_ratio, reduction=reduction, padding=padding,
                 normalize_psf=normalize_psf, enforce_nonnegative=enforce_nonnegative, crop=crop, robust=robust,
                 return_map=return_map, clamp01=clamp01, eps=eps)
