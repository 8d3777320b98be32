"""metrics.lpips_metric on MI355X (reference: metrics/lpips_metric.py:34-117, LPIPSEvaluator over lpips==0.1.4).

LPIPSEvaluator(net='alex' | 'vgg', device)(img_true, img_pred) -> float: the reference's input handling (shape checks,
[C,H,W] promoted to [1,C,H,W], [0,255] -> [0,1] when max > 1.5, [0,1] -> [-1,1] when the values lie in [0,1]) around
the MI355X LPIPS (lpips.py).  Parity unpinned: the lpips package and its pretrained weights are absent here.

Weights: `weights` (an lpips-style state_dict or a path), else the path in $NBP_LPIPS_WEIGHTS_ALEX / _VGG.  A metric
computed with the deterministic synthetic model would not be comparable with the reference's pretrained-weight LPIPS,
so without weights the evaluator raises -- unless `allow_synthetic=True` (or $NBP_LPIPS_ALLOW_SYNTHETIC=1) is given
explicitly, and then `synthetic` is True on the evaluator.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from ..lpips import LPIPS

__all__ = ["LPIPSEvaluator"]


class LPIPSEvaluator:
    """lpips_metric.py:34-117: callable average LPIPS distance over two image batches."""

    def __init__(self, net: str = "alex", device=None, weights=None, allow_synthetic: Optional[bool] = None) -> None:
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        if weights is None:
            weights = os.environ.get(f"NBP_LPIPS_WEIGHTS_{net.upper()}") or None
        if allow_synthetic is None:
            allow_synthetic = os.environ.get("NBP_LPIPS_ALLOW_SYNTHETIC") == "1"
        if weights is None and not allow_synthetic:
            raise RuntimeError(f"LPIPS metric (net={net!r}): pretrained weights are required (pass weights=<lpips "
                               f"state_dict or path> or set NBP_LPIPS_WEIGHTS_{net.upper()}); the offline synthetic "
                               "model gives numbers not comparable with lpips 0.1.4 -- opt in with allow_synthetic=True")
        self.synthetic = weights is None
        self.loss_fn = LPIPS(net=net, weights=weights)
        self.loss_fn.eval()

    @staticmethod
    def _to_minus1_1(x: torch.Tensor) -> torch.Tensor:
        """lpips_metric.py:96-105."""
        if x.numel() == 0:
            return x
        mx, mn = float(x.max().item()), float(x.min().item())
        if mx > 1.5:  # treat as [0, 255]
            x = x / 255.0
        if mn >= 0.0 and mx <= 1.0:
            x = x * 2.0 - 1.0
        return x

    def __call__(self, img_true: torch.Tensor, img_pred: torch.Tensor) -> float:
        if img_true.shape != img_pred.shape:
            raise ValueError(f"Input shapes must match exactly, got {img_true.shape=} and {img_pred.shape=}.")
        if img_true.ndim not in (3, 4):
            raise ValueError(f"Inputs must be 3D (C,H,W) or 4D (N,C,H,W) tensors, received ndim={img_true.ndim}.")
        if img_true.ndim == 3:
            img_true, img_pred = img_true.unsqueeze(0), img_pred.unsqueeze(0)
        img_true = img_true.to(self.device, dtype=torch.float32)
        img_pred = img_pred.to(self.device, dtype=torch.float32)
        with torch.no_grad():
            d = self.loss_fn(self._to_minus1_1(img_pred).contiguous(), self._to_minus1_1(img_true).contiguous())
        return float(d.mean().item())


_CACHE: Dict[Tuple[str, str], LPIPSEvaluator] = {}


def evaluator(net: str, device: Optional[str]) -> LPIPSEvaluator:
    """One evaluator per (net, device): the reference rebuilds lpips.LPIPS on every lpips_distance call; the MI355X
    build keeps the device weights resident (same values)."""
    key = (net, str(device))
    if key not in _CACHE:
        _CACHE[key] = LPIPSEvaluator(net=net, device=device)
    return _CACHE[key]
