"""metrics.ssim on MI355X (reference: metrics/ssim.py:341-377 calculate_ssim -> torchmetrics 1.2.0
StructuralSimilarityIndexMeasure, gaussian 11 / sigma 1.5, k1 0.01, k2 0.03, elementwise mean).

torchmetrics is a third-party dependency absent here: its published algorithm is restated (parity unpinned,
SURVEY §8c): normalised Gaussian window, reflect padding of k//2, the five filtered maps, NO variance clamp and NO
eps, the SSIM map's k//2 border cropped, mean over C x H' x W' per image, mean over images.  Runs as
nbp_ssim_linear(clamp_var = 0, eps = 0, crop = 1).  The evaluator's input alignment (ssim.py:138-167, 258-287) runs
on the device too: resize_policy 'center_crop' (index arithmetic on views), 'resize' (the prediction resampled to the
target's size, F.interpolate bilinear / bicubic, align_corners=False: nbp_resize_planes) and color_space 'y' (BT.601
luma: nbp_luma_bt601), pinned by the reference's own helpers (tests/golden/ssim_align.npz).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _lib
from .._lib import call
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


def _ensure_batch_dim(x: torch.Tensor) -> torch.Tensor:
    """ssim.py:47-57."""
    if x.ndim == 4:
        return x
    if x.ndim == 3:
        return x.unsqueeze(0)
    raise ValueError(f"SSIM expects tensors with 3 (C,H,W) or 4 (N,C,H,W) dimensions. Received shape {tuple(x.shape)}.")


def _to_luma_bt601(x: torch.Tensor) -> torch.Tensor:
    """ssim.py:119-131: 0.2989 R + 0.5870 G + 0.1140 B -> [N,1,H,W] (nbp_luma_bt601)."""
    if x.shape[1] != 3:
        raise ValueError(f"color_space='y' expects 3-channel RGB input, got C={x.shape[1]}.")
    x = x.contiguous()
    N, _, H, W = x.shape
    y = torch.empty(N, 1, H, W, device=x.device)
    call("luma_bt601", x, N, H, W, y)
    return y


def _resize(x: torch.Tensor, size, mode: str) -> torch.Tensor:
    """F.interpolate(x, size, mode, align_corners=False) for mode 'bilinear' / 'bicubic' (nbp_resize_planes)."""
    if mode not in ("bilinear", "bicubic"):
        raise ValueError(f"resize_mode must be 'bilinear' or 'bicubic', got {mode!r}")
    x = x.contiguous()
    N, C, Hi, Wi = x.shape
    Ho, Wo = int(size[0]), int(size[1])
    y = torch.empty(N, C, Ho, Wo, device=x.device)
    call("resize_planes", x, N * C, Hi, Wi, Ho, Wo, int(mode == "bicubic"), y)
    return y


def _align_pair(target: torch.Tensor, prediction: torch.Tensor, policy: Optional[str], mode: str = "bilinear"):
    """ssim.py:134-167: equal sizes required without a policy; 'resize' resamples the prediction to the target's
    size; 'center_crop' crops both to the common size around their centres."""
    if policy is None:
        if target.shape[-2:] != prediction.shape[-2:]:
            raise ValueError("SSIM requires equal spatial dimensions when no resize_policy is set. "
                             f"Got target={target.shape[-2:]}, prediction={prediction.shape[-2:]}")
        return target, prediction
    if policy == "resize":
        return target, _resize(prediction, target.shape[-2:], mode)
    if policy == "center_crop":
        h = min(target.shape[-2], prediction.shape[-2])
        w = min(target.shape[-1], prediction.shape[-1])

        def _crop(x):
            H, W = x.shape[-2:]
            top, left = max((H - h) // 2, 0), max((W - w) // 2, 0)
            return x[:, :, top:top + h, left:left + w].contiguous()

        return _crop(target), _crop(prediction)
    raise ValueError(f"Unknown resize_policy '{policy}'. Use None, 'resize', or 'center_crop'.")


def calculate_ssim(img_true: torch.Tensor, img_pred: torch.Tensor, data_range: float, *, kernel_size: int = 11,
                   sigma: float = 1.5, k1: float = 0.01, k2: float = 0.03, win_size: Optional[int] = None,
                   color_space: str = "rgb", resize_policy: Optional[str] = None, resize_mode: str = "bilinear",
                   domain: Optional[str] = None) -> float:
    if data_range <= 0:
        raise ValueError(f"data_range must be positive, received {data_range}.")
    if win_size is not None:
        kernel_size = int(win_size)
    t = _ensure_batch_dim(img_true)
    p = _ensure_batch_dim(img_pred)
    if t.shape[:2] != p.shape[:2]:
        raise ValueError("SSIM requires the same batch size and channel count for target and prediction. "
                         f"Got target={t.shape}, prediction={p.shape}.")
    # the reference's _prepare_inputs (ssim.py:269-271) moves both to the evaluator's device as float32: CPU tensors
    # are accepted and moved to the GPU the kernels run on (the first CUDA input's device, else the current one)
    if not torch.cuda.is_available():
        raise _lib.NBPError("calculate_ssim runs on the GPU (HIP kernels); no GPU is visible and there is no CPU path")
    dev = t.device if t.is_cuda else (p.device if p.is_cuda else torch.device("cuda", torch.cuda.current_device()))
    t, p = t.to(dev, torch.float32), p.to(dev, torch.float32)
    t, p = _align_pair(t, p, resize_policy, resize_mode)
    if color_space == "y":
        if t.shape[1] == 3:
            t, p = _to_luma_bt601(t), _to_luma_bt601(p)
        elif t.shape[1] != 1:
            raise ValueError(f"color_space='y' expects inputs with 1 or 3 channels, got C={t.shape[1]}.")
    elif color_space != "rgb":
        raise ValueError(f"Unsupported color_space '{color_space}'. Use 'rgb' or 'y'.")
    kernel_size = _valid_kernel_size(t.shape[-2], t.shape[-1], kernel_size)
    c1 = (k1 * float(data_range)) ** 2
    c2 = (k2 * float(data_range)) ** 2
    planes = ssim_plane_means(p, t, kernel_size, sigma, True, c1, c2, 0.0, "reflect", clamp_var=False, crop=True)
    return float(planes.mean(dim=1).mean().item())
