"""NewBP_model.newbp_layer on MI355X (reference: NewBP_model/newbp_layer.py).

Same names, arguments and error behaviour: NewBPFunction, NewBPLayer (deprecated input-side operator),
CrosstalkPSF (the Scenario-B loss-side PSF), build_psf_kernels.  The depthwise PSF convolution and its
conv_transpose2d adjoint run as HIP kernels (nbp_dwconv_nchw_fwd / _bwd_zero); the per-kernel normalisation is
the library's bit-exact host routine.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from .._lib import call

# corner, edge, centre of the fixed 3x3 tables (newbp_layer.py:44-79, 140-164)
_TABLES = {"P2": (0.0100, 0.0200, 0.8800), "R": (0.0117, 0.0233, 0.8600),
           "G": (0.0100, 0.0200, 0.8800), "B": (0.0083, 0.0167, 0.9000)}


def _table(name: str) -> torch.Tensor:
    c, e, m = _TABLES[name]
    return torch.tensor([[c, e, c], [e, m, e], [c, e, c]], dtype=torch.float32).view(1, 1, 3, 3)


# "Stressed" RGB crosstalk family (R > G > B leakage) — a BUILD artefact, not a reference table: the reference only
# describes it (README.md:24,64,214).  S1/S2/S3 leak 1.5x/2x/2.5x of B2's off-centre mass (R .14, G .12,
# B .10) with B2's edge:corner = 2:1 split: corner = leak / 12, edge = leak / 6, centre = 1 - leak.
STRESSED = {f"S{i}": tuple(round(f * l, 6) for l in (0.14, 0.12, 0.10)) for i, f in ((1, 1.5), (2, 2.0), (3, 2.5))}


def _stressed(spec: str, leak: float) -> torch.Tensor:
    c, e, m = leak / 12.0, leak / 6.0, 1.0 - leak
    return torch.tensor([[c, e, c], [e, m, e], [c, e, c]], dtype=torch.float32).view(1, 1, 3, 3)


def build_psf_kernels(mode: str, kernel_spec: str = "P2") -> torch.Tensor:
    """newbp_layer.py:129-173: mono/P2 -> [1,1,3,3]; rgb/B2 -> [3,1,3,3]."""
    if mode not in {"mono", "rgb"}:
        raise ValueError("mode must be 'mono' or 'rgb'")
    if mode == "mono":
        if kernel_spec != "P2":
            raise ValueError("mono mode expects kernel_spec 'P2'")
        return _table("P2")
    if kernel_spec in STRESSED:
        return torch.cat([_stressed(kernel_spec, leak) for leak in STRESSED[kernel_spec]], 0)
    if kernel_spec != "B2":
        raise ValueError("rgb mode expects kernel_spec 'B2' (or the stressed family 'S1', 'S2', 'S3')")
    return torch.cat((_table("R"), _table("G"), _table("B")), dim=0)


def normalize_kernels(k: torch.Tensor) -> torch.Tensor:
    """k / clamp_min(k.view(K,-1).sum(1), 1e-12) with torch's CPU fp32 summation order (bit-exact)."""
    src = np.ascontiguousarray(k.detach().to("cpu", torch.float32).numpy().reshape(k.shape[0], -1))
    out = np.empty_like(src)
    rc = _lib.lib().dll.nbp_psf_normalize_host(src.ctypes.data, src.shape[0], src.shape[1], out.ctypes.data)
    if rc != 0:
        raise _lib.NBPError(_lib.lib().dll.nbp_last_error_string().decode())
    return torch.from_numpy(out).view(k.shape).to(k.device)


class _DWConv3x3Fn(torch.autograd.Function):
    """F.conv2d(x, k, padding=1, groups=C) forward; conv_transpose2d(g, k, padding=1, groups=C) backward."""

    @staticmethod
    def forward(ctx, x, k, shared):
        _lib.require_cuda(x, k)
        x = x.contiguous()
        N, C, H, W = x.shape
        kk = k.detach().contiguous()
        y = torch.empty_like(x)
        call("dwconv_nchw_fwd", x, kk, int(shared), y, N, C, H, W, kk.shape[-2], kk.shape[-1], 0, 0)
        ctx.save_for_backward(kk)
        ctx.shared = shared
        return y

    @staticmethod
    def backward(ctx, gy):
        (kk,) = ctx.saved_tensors
        gy = gy.contiguous()
        N, C, H, W = gy.shape
        gx = torch.empty_like(gy)
        call("dwconv_nchw_bwd_zero", gy, kk, int(ctx.shared), gx, N, C, H, W, kk.shape[-2], kk.shape[-1])
        return gx, None, None


class NewBPFunction(torch.autograd.Function):
    """newbp_layer.py:7-21: conv2d forward, conv_transpose2d backward, no kernel gradient (depthwise form)."""

    @staticmethod
    def forward(ctx, input, kernel, padding, groups):
        if padding != (kernel.shape[-1] - 1) // 2 or groups != input.shape[1] or kernel.shape[1] != 1:
            raise NotImplementedError("NewBPFunction on MI355X supports the depthwise same-padding form used by NewBPLayer")
        _lib.require_cuda(input, kernel)
        x = input.contiguous()
        N, C, H, W = x.shape
        kk = kernel.detach().contiguous()
        y = torch.empty_like(x)
        call("dwconv_nchw_fwd", x, kk, 0, y, N, C, H, W, kk.shape[-2], kk.shape[-1], 0, 0)
        ctx.save_for_backward(kk)
        return y

    @staticmethod
    def backward(ctx, grad_outputs):
        (kk,) = ctx.saved_tensors
        g = grad_outputs.contiguous()
        N, C, H, W = g.shape
        gx = torch.empty_like(g)
        call("dwconv_nchw_bwd_zero", g, kk, 0, gx, N, C, H, W, kk.shape[-2], kk.shape[-1])
        return gx, None, None, None


class NewBPLayer(nn.Module):
    """newbp_layer.py:24-85 — deprecated input-side NewBP operator (raises unless deprecated=False)."""

    def __init__(self, in_channels=3, kernel_type="panchromatic", kernel_spec="P2", *, deprecated: bool = True):
        super().__init__()
        self.in_channels = in_channels
        self.kernel_type = kernel_type
        self.kernel_spec = kernel_spec
        self.deprecated = deprecated
        if kernel_spec not in {"P2", "B2"}:
            raise ValueError(f"Unsupported kernel_spec '{kernel_spec}'. Expected 'P2' or 'B2'.")
        if kernel_type not in {"panchromatic", "rgb"}:
            raise ValueError(f"Unsupported kernel_type '{kernel_type}'. Expected 'panchromatic' or 'rgb'.")
        if kernel_type == "rgb" and in_channels != 3:
            raise ValueError("kernel_type 'rgb' requires in_channels to be 3.")
        self.kernel = nn.Parameter(self._build_kernel(), requires_grad=False)

    def _build_kernel(self):
        if self.kernel_type == "panchromatic":
            if self.kernel_spec != "P2":
                raise ValueError("kernel_type 'panchromatic' requires kernel_spec 'P2'.")
            return _table("P2").repeat(self.in_channels, 1, 1, 1)  # un-normalised (:56)
        if self.kernel_spec == "P2":
            raise ValueError("kernel_type 'rgb' requires kernel_spec 'B2'.")
        return torch.cat((_table("R"), _table("G"), _table("B")), dim=0)

    def forward(self, x):
        if self.deprecated:
            raise RuntimeError("Deprecated: use CrosstalkPSF in loss path (Scenario B).")
        padding = (self.kernel.shape[-1] - 1) // 2
        return NewBPFunction.apply(x, self.kernel, padding, self.in_channels)


class CrosstalkPSF(nn.Module):
    """newbp_layer.py:88-126 — fixed PSF used only in the loss graph; `kernel` is a persistent buffer,
    normalised per kernel at construction."""

    def __init__(self, mode: str, kernels: torch.Tensor):
        super().__init__()
        assert mode in {"mono", "rgb"}
        self.mode = mode
        self.register_buffer("kernel", normalize_kernels(kernels.clone()), persistent=True)
        self.kernel: torch.Tensor

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        C = x.shape[1]
        assert C == 3, "CrosstalkPSF expects sRGB inputs (3 channels)."
        k = self.kernel
        if self.mode == "mono":
            assert k.shape == (1, 1, 3, 3), "mono mode expects kernels of shape [1,1,3,3]"
        else:
            assert k.shape == (3, 1, 3, 3), "rgb mode expects kernels of shape [3,1,3,3]"
        return _DWConv3x3Fn.apply(x, k.to(x.dtype), self.mode == "mono")
