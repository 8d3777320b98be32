"""metrics.linear on MI355X (reference: metrics/linear.py) — linear-domain PSNR and SSIM.

Same names, arguments, validation and exception types as the reference; the arithmetic runs in HIP kernels
(metrics.hip): per-sample float64 squared-error sums for PSNR (:140-215) and a separable windowed SSIM with the
reference's padding modes, variance clamp and eps (:218-324).  fp32 inputs (the kernels read fp32; a float64 input is
evaluated in fp32 — the reference's own metric path casts to fp32 for every caller in this repository).
"""
from __future__ import annotations

from functools import lru_cache
from typing import Literal

import torch
from torch import Tensor

from .. import _lib
from .._lib import call, query

__all__ = ["psnr_linear", "ssim_linear"]

_Reduction = Literal["mean", "sum", "none"]
_ChannelAggregate = Literal["mean", "none"]
_PaddingMode = Literal["reflect", "replicate", "circular", "constant"]
_PAD_CODE = {"reflect": 0, "replicate": 1, "circular": 2, "constant": 3}


def _ensure_nchw(pred: Tensor, target: Tensor) -> tuple[Tensor, Tensor]:
    """linear.py _ensure_nchw: type/dtype/device/shape/finiteness checks, [C,H,W] promoted to [1,C,H,W]."""
    if not isinstance(pred, Tensor) or not isinstance(target, Tensor):
        raise TypeError("psnr_linear/ssim_linear expect torch.Tensor inputs.")
    if pred.dtype not in {torch.float32, torch.float64}:
        raise TypeError(f"Expected pred dtype float32/float64, received {pred.dtype}.")
    if target.dtype != pred.dtype:
        raise TypeError("pred and target must share the same dtype.")
    if pred.device != target.device:
        raise ValueError("pred and target must live on the same device.")
    if pred.shape != target.shape:
        raise ValueError(f"pred and target must share identical shape, got {pred.shape} vs {target.shape}.")
    if not torch.isfinite(pred).all():
        raise ValueError("pred contains NaN or Inf values.")
    if not torch.isfinite(target).all():
        raise ValueError("target contains NaN or Inf values.")
    if pred.ndim == 3:
        pred, target = pred.unsqueeze(0), target.unsqueeze(0)
    elif pred.ndim != 4:
        raise ValueError("Inputs must have 3 (C,H,W) or 4 (N,C,H,W) dimensions; "
                         f"received tensor with shape {tuple(pred.shape)}.")
    if pred.shape[0] == 0:
        raise ValueError("Batch dimension cannot be zero.")
    if pred.shape[1] == 0:
        raise ValueError("Channel dimension cannot be zero.")
    if pred.shape[2] == 0 or pred.shape[3] == 0:
        raise ValueError("Spatial dimensions must be strictly positive.")
    return pred.detach(), target.detach()


def _reduce(values: Tensor, reduction: _Reduction) -> Tensor:
    if reduction == "none":
        return values
    if reduction == "mean":
        return values.mean(dim=0)
    if reduction == "sum":
        return values.sum(dim=0)
    raise ValueError(f"Unsupported reduction='{reduction}'. Expected 'mean', 'sum', or 'none'.")


def _f32(t: Tensor) -> Tensor:
    _lib.require_cuda(t)
    return t.to(torch.float32).contiguous()


def psnr_per_sample(pred: Tensor, target: Tensor, data_range: float, eps: float, diff_double: bool) -> Tensor:
    """float64 [N] PSNR of [N, ...] fp32 tensors (inf where mse <= eps) — nbp_psnr."""
    p, t = _f32(pred), _f32(target)
    N = p.shape[0]
    L = p.numel() // N
    ws = torch.empty(query("psnr_workspace_doubles", N, L), dtype=torch.float64, device=p.device)
    out = torch.empty(N, dtype=torch.float64, device=p.device)
    call("psnr", p, t, N, L, float(data_range), float(eps), int(diff_double), ws, None, out)
    return out


def psnr_linear(pred: Tensor, target: Tensor, data_range: float = 1.0, reduction: _Reduction = "mean",
                eps: float = 1e-12) -> Tensor:
    """PSNR in the linear domain (linear.py:140-215): per-sample float64 MSE, 10 log10(range^2 / max(mse, eps)),
    +inf where mse <= eps; batch reduction mean / sum / none."""
    if data_range <= 0:
        raise ValueError(f"`data_range` must be positive, received {data_range}.")
    if eps <= 0:
        raise ValueError(f"`eps` must be positive, received {eps}.")
    pred, target = _ensure_nchw(pred, target)
    return _reduce(psnr_per_sample(pred, target, data_range, eps, diff_double=False), reduction)


@lru_cache(maxsize=None)
def _window_1d(kernel_size: int, sigma: float, gaussian: bool) -> tuple:
    """The normalised separable factor of the reference's float64 2-D window (Gaussian exp(-x^2 / 2 sigma^2) or
    uniform), as a tuple of floats."""
    if gaussian:
        if sigma <= 0:
            raise ValueError("sigma must be positive when gaussian=True.")
        coords = torch.arange(kernel_size, dtype=torch.float64) - (kernel_size - 1) / 2.0
        k = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    else:
        k = torch.ones(kernel_size, dtype=torch.float64)
    return tuple((k / k.sum()).tolist())


def ssim_plane_means(pred: Tensor, target: Tensor, kernel_size: int, sigma: float, gaussian: bool, c1: float,
                     c2: float, eps: float, padding: str, clamp_var: bool, crop: bool) -> Tensor:
    """float64 [N, C] means of the windowed SSIM map — nbp_ssim_linear."""
    p, t = _f32(pred), _f32(target)
    N, C, H, W = p.shape
    win = torch.tensor(_window_1d(int(kernel_size), float(sigma), bool(gaussian)), dtype=torch.float32,
                       device=p.device)
    ws = torch.empty(query("ssim_linear_workspace_floats", N, C, H, W), device=p.device)
    out = torch.empty(N * C, dtype=torch.float64, device=p.device)
    call("ssim_linear", p, t, N, C, H, W, win, int(kernel_size), _PAD_CODE[padding], float(c1), float(c2),
         float(eps), int(clamp_var), int(crop), ws, out)
    return out.view(N, C)


def ssim_linear(pred: Tensor, target: Tensor, data_range: float = 1.0, kernel_size: int = 11, sigma: float = 1.5,
                k1: float = 0.01, k2: float = 0.03, gaussian: bool = True, reduction: _Reduction = "mean",
                channel_aggregate: _ChannelAggregate = "mean", padding: _PaddingMode = "reflect",
                eps: float = 1e-12) -> Tensor:
    """SSIM in the linear domain (linear.py:218-324)."""
    if data_range <= 0:
        raise ValueError(f"`data_range` must be positive, received {data_range}.")
    if eps <= 0:
        raise ValueError(f"`eps` must be positive, received {eps}.")
    if k1 < 0 or k2 < 0:
        raise ValueError("k1 and k2 must be non-negative.")
    if channel_aggregate not in {"mean", "none"}:
        raise ValueError(f"channel_aggregate must be 'mean' or 'none', received {channel_aggregate}.")
    pred, target = _ensure_nchw(pred, target)
    n, c, h, w = pred.shape
    if h < kernel_size or w < kernel_size:
        raise ValueError("Spatial dimensions must be >= kernel_size. "
                         f"Got H={h}, W={w}, kernel_size={kernel_size}.")
    if kernel_size <= 0 or kernel_size % 2 == 0:
        raise ValueError(f"kernel_size must be a positive odd integer; received {kernel_size}.")
    if padding not in _PAD_CODE:
        raise ValueError(f"Unsupported padding mode '{padding}'.")
    c1 = (k1 * float(data_range)) ** 2
    c2 = (k2 * float(data_range)) ** 2
    per_channel = ssim_plane_means(pred, target, kernel_size, sigma, gaussian, c1, c2, eps, padding,
                                   clamp_var=True, crop=False)
    per_image = per_channel.mean(dim=1) if channel_aggregate == "mean" else per_channel
    return _reduce(per_image.to(pred.dtype), reduction)
