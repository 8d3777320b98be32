"""metrics.ssim on MI355X (reference: metrics/ssim.py:341-377 calculate_ssim -> torchmetrics 1.2.0
StructuralSimilarityIndexMeasure, gaussian 11 / sigma 1.5, k1 0.01, k2 0.03, elementwise mean).

torchmetrics is a third-party dependency absent here: its published algorithm is restated (parity unpinned,
SURVEY §8c): normalised Gaussian window, reflect padding of k//2, the five filtered maps, NO variance clamp and NO
eps, the SSIM map's k//2 border cropped, mean over C x H' x W' per image, mean over images.  Runs as
nbp_ssim_linear(clamp_var = 0, eps = 0, crop = 1).  Only the rgb colour space without resizing is supported (the
reference's default); other options raise NotImplementedError.
"""
from __future__ import annotations

from typing import Optional

import torch

from .linear import ssim_plane_means

__all__ = ["calculate_ssim"]


def _valid_kernel_size(height: int, width: int, kernel_size: int) -> int:
    """metrics/ssim.py:74-89: an odd window no larger than the smaller image side."""
    k = int(kernel_size)
    if k <= 0:
        raise ValueError(f"kernel_size must be positive, received {kernel_size}.")
    if k % 2 == 0:
        k -= 1
    k = max(1, min(k, height, width))
    if k % 2 == 0:
        k -= 1
    if k < 1:
        raise ValueError(f"kernel_size cannot be adjusted to a valid value for shape {(height, width)}.")
    return k


def calculate_ssim(img_true: torch.Tensor, img_pred: torch.Tensor, data_range: float, *, kernel_size: int = 11,
                   sigma: float = 1.5, k1: float = 0.01, k2: float = 0.03, win_size: Optional[int] = None,
                   color_space: str = "rgb", resize_policy: Optional[str] = None, resize_mode: str = "bilinear",
                   domain: Optional[str] = None) -> float:
    if data_range <= 0:
        raise ValueError(f"data_range must be positive, received {data_range}.")
    if win_size is not None:
        kernel_size = int(win_size)
    if color_space != "rgb" or resize_policy is not None:
        raise NotImplementedError("calculate_ssim on MI355X supports color_space='rgb' without resizing")
    t = img_true if img_true.dim() == 4 else img_true.unsqueeze(0)
    p = img_pred if img_pred.dim() == 4 else img_pred.unsqueeze(0)
    if t.shape != p.shape:
        raise ValueError("SSIM requires the same batch size and channel count for target and prediction. "
                         f"Got target={t.shape}, prediction={p.shape}.")
    kernel_size = _valid_kernel_size(t.shape[-2], t.shape[-1], kernel_size)
    c1 = (k1 * float(data_range)) ** 2
    c2 = (k2 * float(data_range)) ** 2
    planes = ssim_plane_means(p, t, kernel_size, sigma, True, c1, c2, 0.0, "reflect", clamp_var=False, crop=True)
    return float(planes.mean(dim=1).mean().item())
