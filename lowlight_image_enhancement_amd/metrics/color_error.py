"""metrics.color_error on MI355X (reference: metrics/color_error.py) — CIEDE2000 maps and summaries.

deltaE2000_map (:235-267) -> _deltaE00_lab_map (:105-210) runs as one HIP kernel per pixel (color.hip:
kornia-0.6.12 rgb_to_lab restated + the reference's metric-form CIEDE2000).  The percentile summaries use
torch.quantile on the device-resident map (a sort; statistics plumbing, not a reimplemented reference kernel);
edge_deltaE2000's Sobel magnitude of L is nbp_sobel_mag.
"""
from __future__ import annotations

import warnings
from typing import Dict, Iterable, Literal, Tuple

import torch
from torch import Tensor

from .. import _lib
from .._lib import call

_WHITEPOINT = Literal["D65-2", "D50-2"]

__all__ = ["deltaE2000_map", "deltaE2000_summary", "edge_deltaE2000"]


def _ensure_nchw(rgb1: Tensor, rgb2: Tensor) -> Tuple[Tensor, Tensor, bool]:
    """color_error.py:33-66."""
    if not isinstance(rgb1, Tensor) or not isinstance(rgb2, Tensor):
        raise TypeError("deltaE2000 functions expect torch.Tensor inputs.")
    if rgb1.shape != rgb2.shape:
        raise ValueError(f"pred_srgb and target_srgb must share identical shape, got {tuple(rgb1.shape)} vs "
                         f"{tuple(rgb2.shape)}.")
    if rgb1.device != rgb2.device:
        raise ValueError("pred_srgb and target_srgb must reside on the same device.")
    was_3d = False
    if rgb1.ndim == 3:
        rgb1, rgb2, was_3d = rgb1.unsqueeze(0), rgb2.unsqueeze(0), True
    elif rgb1.ndim != 4:
        raise ValueError("Expected tensors with 3 (C,H,W) or 4 (N,C,H,W) dimensions; "
                         f"received tensor with shape {tuple(rgb1.shape)}.")
    if rgb1.shape[1] != 3:
        raise ValueError(f"sRGB inputs must have 3 channels. Received {rgb1.shape[1]}.")
    if not torch.isfinite(rgb1).all():
        raise ValueError("pred_srgb contains NaN or Inf values.")
    if not torch.isfinite(rgb2).all():
        raise ValueError("target_srgb contains NaN or Inf values.")
    return rgb1.detach(), rgb2.detach(), was_3d


def _whitepoint_warning(whitepoint):
    if whitepoint == "D50-2":
        warnings.warn("deltaE2000_map called with whitepoint='D50-2'. Ensure inputs were Bradford-adapted from D65 to "
                      "D50 upstream (CSS Color 4). This function does not perform chromatic adaptation internally.",
                      RuntimeWarning)


def _f32(t: Tensor) -> Tensor:
    _lib.require_cuda(t)
    return t.to(torch.float32).contiguous()


@torch.no_grad()
def deltaE2000_map(pred_srgb: Tensor, target_srgb: Tensor, *, kL: float = 1.0, kC: float = 1.0, kH: float = 1.0,
                   whitepoint: _WHITEPOINT = "D65-2", eps: float = 1e-12) -> Tensor:
    """ΔE00 map [N,H,W] (or [H,W] for 3-D inputs) between sRGB images in [0, 1]."""
    if eps <= 0:
        raise ValueError(f"`eps` must be positive, received {eps}.")
    pred, target, was_3d = _ensure_nchw(pred_srgb, target_srgb)
    _whitepoint_warning(whitepoint)
    pred, target = _f32(pred), _f32(target)
    N, _, H, W = pred.shape
    out = torch.empty(N, H, W, device=pred.device)
    call("de00_metric_map", pred, target, N, H, W, float(kL), float(kC), float(kH), float(eps), out)
    return out.squeeze(0) if was_3d else out


def _compute_percentiles(values: Tensor, percentiles: Iterable[float]) -> Dict[str, float]:
    stats: Dict[str, float] = {}
    flat = values.view(-1)
    if flat.numel() == 0:
        for p in percentiles:
            stats[f"p{int(p)}"] = float("nan")
        return stats
    qs = []
    for p in percentiles:
        q = float(p)
        if not 0.0 <= q <= 100.0:
            raise ValueError(f"Percentile values must lie within [0, 100]; received {q}.")
        qs.append(q / 100.0)
    quant = torch.quantile(flat, torch.tensor(qs, device=flat.device, dtype=flat.dtype))
    for i, p in enumerate(percentiles):
        stats[f"p{int(p)}"] = float(quant[i].item())
    return stats


@torch.no_grad()
def deltaE2000_summary(pred_srgb: Tensor, target_srgb: Tensor, *, percentiles: Tuple[float, ...] = (50.0, 95.0),
                       **kwargs) -> Dict[str, float]:
    """Mean (of per-image means) and percentiles of the ΔE00 map (color_error.py:270-293)."""
    de_map = deltaE2000_map(pred_srgb, target_srgb, **kwargs)
    flat = de_map.view(de_map.shape[0], -1) if de_map.dim() == 3 else de_map.view(1, -1)
    summary: Dict[str, float] = {"mean": float(flat.mean(dim=1).mean().item())}
    summary.update(_compute_percentiles(flat.reshape(-1), percentiles))
    return summary


@torch.no_grad()
def edge_deltaE2000(pred_srgb: Tensor, target_srgb: Tensor, *, method: str = "sobel", q: float = 0.85,
                    **kwargs) -> Dict[str, float]:
    """ΔE00 restricted to pixels whose Sobel |grad L| is >= the per-image q-quantile (color_error.py:305-344)."""
    if method != "sobel":
        raise ValueError(f"Unsupported edge detection method '{method}'. Currently only 'sobel' is available.")
    if not 0.0 < q < 1.0:
        raise ValueError(f"q must lie within (0,1); received {q}.")
    de_map = deltaE2000_map(pred_srgb, target_srgb, **kwargs)
    pred, _, _ = _ensure_nchw(pred_srgb, target_srgb)
    pred = _f32(pred)
    N, _, H, W = pred.shape
    lab = torch.empty_like(pred)
    call("rgb_to_lab", pred, N, H, W, lab)
    grad = torch.empty(N, 1, H, W, device=pred.device)
    call("sobel_mag", lab, N, H, W, grad)
    if de_map.ndim == 2:
        de_map = de_map.unsqueeze(0)
    de_map = de_map.unsqueeze(1)
    threshold = torch.quantile(grad.view(N, -1), q, dim=1, keepdim=True)
    mask = grad >= threshold.view(-1, 1, 1, 1)
    vals = de_map[mask.expand_as(de_map)]
    if vals.numel() == 0:
        return {"mean": float("nan"), "p95": float("nan")}
    return {"mean": float(vals.mean().item()), "p95": float(torch.quantile(vals, 0.95).item())}
