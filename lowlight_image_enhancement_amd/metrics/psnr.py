"""metrics.psnr on MI355X (reference: metrics/psnr.py:18-67) — calculate_psnr over the whole tensor with the
difference taken in float64 (nbp_psnr, diff_double = 1); +inf when the mse is within 1e-12 of zero."""
from __future__ import annotations

import torch

from .linear import psnr_per_sample

__all__ = ["calculate_psnr"]


def calculate_psnr(img_true: torch.Tensor, img_pred: torch.Tensor, data_range: float) -> float:
    if img_true.shape != img_pred.shape:
        raise ValueError(f"Input shapes must match exactly, got {img_true.shape=} and {img_pred.shape=}.")
    if data_range <= 0:
        raise ValueError(f"`data_range` must be positive, received {data_range}.")
    p = psnr_per_sample(img_true.reshape(1, -1), img_pred.reshape(1, -1), data_range, 1e-12, diff_double=True)
    return float(p.item())
