"""basicsr.metrics.lowlight_metrics validation helpers on MI355X (reference:
NAFNet_base/basicsr/metrics/lowlight_metrics.py:211-272): thin wrappers over metrics.psnr / metrics.ssim /
metrics.color_error exactly as the reference composes them (fp32 casts, clamp01 before ΔE00)."""
from __future__ import annotations

from typing import Literal, Optional

import torch

from .color_error import deltaE2000_summary, edge_deltaE2000
from .psnr import calculate_psnr
from .ssim import calculate_ssim

__all__ = ["linear_psnr", "linear_ssim", "lpips_distance", "deltae2000_mean", "deltae2000_p95", "edge_deltae2000_mean"]


def linear_psnr(pred: torch.Tensor, target: torch.Tensor, *, data_range: float = 1.0) -> float:
    return calculate_psnr(target.to(torch.float32), pred.to(torch.float32), data_range=data_range)


def linear_ssim(pred: torch.Tensor, target: torch.Tensor, *, data_range: float = 1.0) -> float:
    return calculate_ssim(target.to(torch.float32), pred.to(torch.float32), data_range=data_range)


def lpips_distance(pred: torch.Tensor, target: torch.Tensor, *, net: str = "vgg", device: Optional[str] = None) -> float:
    """lowlight_metrics.py:223-226: LPIPSEvaluator(net, device)(target, pred)."""
    from .lpips_metric import evaluator
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    return evaluator(net, dev)(target.to(dev), pred.to(dev))


def deltae2000_mean(pred: torch.Tensor, target: torch.Tensor, *,
                    whitepoint: Literal["D65-2", "D50-2"] = "D65-2") -> float:
    return deltaE2000_summary(pred.clamp(0.0, 1.0), target.clamp(0.0, 1.0), whitepoint=whitepoint,
                              percentiles=(95.0,))["mean"]


def deltae2000_p95(pred: torch.Tensor, target: torch.Tensor, *,
                   whitepoint: Literal["D65-2", "D50-2"] = "D65-2") -> float:
    return deltaE2000_summary(pred.clamp(0.0, 1.0), target.clamp(0.0, 1.0), whitepoint=whitepoint,
                              percentiles=(95.0,))["p95"]


def edge_deltae2000_mean(pred: torch.Tensor, target: torch.Tensor, *,
                         whitepoint: Literal["D65-2", "D50-2"] = "D65-2", q: float = 0.85) -> float:
    return edge_deltaE2000(pred.clamp(0.0, 1.0), target.clamp(0.0, 1.0), whitepoint=whitepoint, q=q)["mean"]
