"""NewBP_model.losses on MI355X (reference: NewBP_model/losses.py).

Same class/function names, constructor arguments, term order and return values as the reference; every term's
forward and backward runs as HIP kernels (include/nbp.h): L1 / Charbonnier (nbp_pix_loss_*), SSIM
(nbp_ssim_loss_*), the physics-consistency L1 with the crosstalk PSF (nbp_phys_l1_*), exposure alignment
(nbp_align_exposure), ΔE00 (nbp_de00_loss_*).  Scalars stay on the device; the upstream gradient is read from device
memory.

The VGG19 perceptual term runs as implicit-GEMM MFMA convs (vgg.py: fp32 like the reference's trunk, or 16-bit
operands under autocast / the trainer's 16-bit modes); LPIPS is lpips.py.
"""
from __future__ import annotations

import warnings
from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from .. import _lib
from .. import vgg as _vgg
from ..lpips import LPIPS
from .._lib import call, query
from .newbp_layer import CrosstalkPSF


def _resolve_device(device: Union[str, torch.device]) -> torch.device:
    """losses.py:20-29."""
    if isinstance(device, torch.device):
        return device
    if isinstance(device, str):
        if device == "auto":
            return torch.device("cuda" if torch.cuda.is_available() else "cpu")
        return torch.device(device)
    raise TypeError(f"Unsupported device spec: {device!r}")


# ---------------------------------------------------------------- autograd wrappers over the C-ABI
class _PixLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, mode, eps, clamp_a, clamp_b):
        _lib.require_cuda(a, b)
        if a.shape != b.shape:
            raise ValueError(f"shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
        a, b = a.contiguous(), b.contiguous()
        n = a.numel()
        ws = torch.empty(query("pix_workspace_doubles", n), dtype=torch.float64, device=a.device)
        loss = torch.empty((), device=a.device)
        call("pix_loss_fwd", a, b, n, mode, eps, clamp_a, clamp_b, ws, loss)
        ctx.save_for_backward(a, b)
        ctx.args = (mode, eps, clamp_a, clamp_b)
        return loss

    @staticmethod
    def backward(ctx, up):
        a, b = ctx.saved_tensors
        mode, eps, ca, cb = ctx.args
        up = up.contiguous()
        ga = gb = None
        if ctx.needs_input_grad[0]:
            ga = torch.empty_like(a)
            call("pix_loss_bwd", a, b, a.numel(), mode, eps, ca, cb, up, ga)
        if ctx.needs_input_grad[1]:
            gb = torch.empty_like(b)
            call("pix_loss_bwd", b, a, b.numel(), mode, eps, cb, ca, up, gb)
        return ga, gb, None, None, None, None


def l1_loss(a, b, clamp01=False):
    return _PixLossFn.apply(a, b, 0, 0.0, bool(clamp01), bool(clamp01))


def charbonnier_loss(a, b, eps=1e-12):
    """NAFNet_base/basicsr/models/losses/losses.py:29-31 (mean reduction)."""
    return _PixLossFn.apply(a, b, 1, float(eps), False, False)


_SSIM_REDUCTION = {"mean": 0, "sum": 1, "none": 2}


class _SSIMLossFn(torch.autograd.Function):
    """kornia 0.6.12 ssim_loss: clamp((1 - ssim(x, y)) / 2, 0, 1) reduced by 'mean' / 'sum' / 'none' (the map).  The
    map is symmetric in (x, y), so d/dy is the kernel pair with the inputs swapped (a second forward, made only when
    y needs a gradient, that writes the coefficients only: no loss, no map)."""

    @staticmethod
    def forward(ctx, x, y, window, max_val, clamp_in, reduction):
        _lib.require_cuda(x, y)
        if x.shape != y.shape or x.dim() != 4:
            raise ValueError("SSIMLoss expects two [N,C,H,W] tensors of the same shape")
        x, y = x.contiguous(), y.contiguous()
        N, C, H, W = x.shape
        red = _SSIM_REDUCTION[reduction]
        loss = torch.empty((), device=x.device) if red != 2 else None
        lmap = torch.empty_like(x) if red == 2 else None
        wsx = wsy = None
        want_x, want_y = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        wsx = torch.empty(query("ssim_workspace_floats", x.numel()), device=x.device)
        call("ssim_loss_fwd", x, y, N, C, H, W, window, float(max_val), clamp_in, int(want_x), red, wsx, loss, lmap)
        if want_y:
            wsy = torch.empty(query("ssim_workspace_floats", x.numel()), device=x.device)
            call("ssim_loss_fwd", y, x, N, C, H, W, window, float(max_val), clamp_in, 1, red, wsy, None, None)
        ctx.save_for_backward(x, y, wsx, wsy)
        ctx.clamp_in, ctx.red = clamp_in, red
        return loss if red != 2 else lmap

    @staticmethod
    def backward(ctx, up):
        x, y, wsx, wsy = ctx.saved_tensors
        N, C, H, W = x.shape
        up = up.float().contiguous()
        us, um = (None, up) if ctx.red == 2 else (up.view(1), None)
        gx = gy = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            call("ssim_loss_bwd", x, y, N, C, H, W, ctx.clamp_in, us, um, wsx, gx)
        if ctx.needs_input_grad[1]:
            gy = torch.empty_like(y)
            call("ssim_loss_bwd", y, x, N, C, H, W, ctx.clamp_in, us, um, wsy, gy)
        return gx, gy, None, None, None, None


def _ratio_array(ratio, ref: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Broadcast the exposure ratio against ref [N,C,H,W] following losses.py:195-203 (float -> tensor,
    0-d -> [1], 1-d -> [B,1,1,1]); returns ([N*C] per-plane array, 0) or (full [N,C,H,W] map, 1)."""
    N, C, H, W = ref.shape
    if not torch.is_tensor(ratio):
        return torch.full((N * C,), float(ratio), device=ref.device, dtype=torch.float32), 0
    r = ratio.to(device=ref.device, dtype=torch.float32)
    if r.dim() == 0:
        r = r.view(1)
    if r.dim() == 1:
        r = r.view(-1, 1, 1, 1)
    try:
        shape = torch.broadcast_shapes(r.shape, ref.shape)
    except RuntimeError:
        shape = None
    if shape is None or tuple(shape) != tuple(ref.shape):
        raise ValueError(f"exposure ratio of shape {tuple(ratio.shape)} does not broadcast to {tuple(ref.shape)}")
    if r.dim() == 4 and r.shape[2] == 1 and r.shape[3] == 1:
        return r.expand(N, C, 1, 1).contiguous().view(-1), 0
    return r.expand(N, C, H, W).contiguous(), 1


class _PhysL1Fn(torch.autograd.Function):
    """mean |PSF(clamp?(bhat)) - clamp?(clamp?(a)*ratio)| ; pad 0 = zero (sRGB loss), 1 = replicate (raw loss)."""

    @staticmethod
    def forward(ctx, bhat, a, ratio_arr, ratio_full, k, k_shared, pad_mode, clamp_bhat, clamp_a_in, clamp_align):
        _lib.require_cuda(bhat, a, k)
        if bhat.shape != a.shape:
            raise ValueError(f"shape mismatch {tuple(bhat.shape)} vs {tuple(a.shape)}")
        bhat, a = bhat.contiguous(), a.contiguous()
        N, C, H, W = bhat.shape
        kk = k.detach().contiguous()
        ws = torch.empty(query("phys_l1_workspace_doubles", N, C, H, W), dtype=torch.float64, device=bhat.device)
        loss = torch.empty((), device=bhat.device)
        sign = torch.empty_like(bhat) if (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]) else None
        call("phys_l1_fwd", bhat, a, ratio_arr, ratio_full, kk, k_shared, N, C, H, W, kk.shape[-2], kk.shape[-1],
             pad_mode, clamp_bhat, clamp_a_in, clamp_align, ws, loss, sign)
        ctx.save_for_backward(sign, bhat, kk, a, ratio_arr)
        ctx.args = (k_shared, pad_mode, clamp_bhat, clamp_a_in, clamp_align, ratio_full)
        return loss

    @staticmethod
    def backward(ctx, up):
        sign, bhat, kk, a, ratio_arr = ctx.saved_tensors
        k_shared, pad_mode, clamp_bhat, clamp_a_in, clamp_align, ratio_full = ctx.args
        N, C, H, W = bhat.shape
        up = up.float().contiguous().view(1)
        g = ga = None
        if ctx.needs_input_grad[0]:
            g = torch.empty_like(bhat)
            call("phys_l1_bwd", sign, bhat, kk, k_shared, up, N, C, H, W, kk.shape[-2], kk.shape[-1], pad_mode,
                 clamp_bhat, g)
        if ctx.needs_input_grad[1]:  # the short exposure's gradient (plain autograd in the reference)
            ga = torch.empty_like(a)
            call("phys_a_bwd", sign, a, ratio_arr, ratio_full, N, C, C, H, W, clamp_a_in, clamp_align, up, ga)
        return g, ga, None, None, None, None, None, None, None, None


# ---------------------------------------------------------------- public classes (reference names)
class _PerceptualFn(torch.autograd.Function):
    """mean/sum of (VGG(prep(gen)) - VGG(prep(tgt)))^2 (or |.|); d/d gen through the frozen stack (vgg.py)."""

    @staticmethod
    def forward(ctx, gen, tgt, module, dt):
        _lib.require_cuda(gen, tgt)
        if gen.shape != tgt.shape:
            raise ValueError(f"PerceptualLoss: shape mismatch {tuple(gen.shape)} vs {tuple(tgt.shape)}")
        stack = module.stack(gen.device, dt)
        want, want_t = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        with torch.no_grad():
            ft, tape_t, _ = stack.forward(_vgg.prep_input(tgt.detach(), dtype=stack.dtype), save=want_t)
            fg, tape, _ = stack.forward(_vgg.prep_input(gen.detach(), dtype=stack.dtype), save=want)
        n = fg.numel()
        mode = 0 if module.use_mse else 1
        scale = 1.0 / n if module.reduction == "mean" else 1.0
        ws = torch.empty(query("feat_dist_workspace_doubles", n), dtype=torch.float64, device=gen.device)
        out = torch.empty((), device=gen.device)
        call("feat_dist_fwd", fg, ft, n, mode, scale, ws, out, stack.dtype)
        if want or want_t:
            ctx.tape, ctx.tape_t, ctx.fg, ctx.ft, ctx.stack = tape, tape_t, fg, ft, stack
            ctx.mode, ctx.scale = mode, scale
            ctx.save_for_backward(gen.detach(), tgt.detach())
        return out

    @staticmethod
    def backward(ctx, up):
        gen, tgt = ctx.saved_tensors
        up = up.float().contiguous().view(1)
        n = ctx.fg.numel()
        dg = dt_ = None
        if ctx.needs_input_grad[0]:
            d = torch.empty_like(ctx.fg)
            call("feat_dist_bwd", ctx.fg, ctx.ft, n, ctx.mode, float(ctx.scale), 1, up, d, ctx.stack.dtype)
            dg = _vgg.input_grad(ctx.stack.backward(ctx.tape, d), gen)
        if ctx.needs_input_grad[1]:  # MSE / L1 are symmetric: the distance gradient with the features swapped
            d = torch.empty_like(ctx.ft)
            call("feat_dist_bwd", ctx.ft, ctx.fg, n, ctx.mode, float(ctx.scale), 1, up, d, ctx.stack.dtype)
            dt_ = _vgg.input_grad(ctx.stack.backward(ctx.tape_t, d), tgt)
        ctx.tape = ctx.tape_t = ctx.fg = ctx.ft = None
        return dg, dt_, None, None


class PerceptualLoss(nn.Module):
    """losses.py:32-69 — clamp01 -> ImageNet mean/std -> vgg19.features[:36] (through relu5_4) for both images ->
    MSE (use_mse) or L1, reduction 'mean' / 'sum'.  The conv stack is implicit-GEMM MFMA (vgg.py).
    `weights`: None (deterministic synthetic VGG19 — the ImageNet download is unavailable offline), a state_dict of
    vgg19 (`features.N.*` or `N.*` keys) or a checkpoint path (loaded with weights_only=True).  `precision`: the trunk's
    storage / operand type: "auto" (default: fp32 like the reference's `.float()` trunk, fp16 / bf16 inside an enabled
    CUDA autocast region), or "fp32", "bf16", "fp16" explicitly (fp16 wants loss scaling, as NBPTrainer's fp16 mode
    applies)."""

    def __init__(self, device: Union[str, torch.device] = "cuda", use_mse: bool = True, reduction: str = "mean",
                 weights=None, precision: str = "auto"):
        super().__init__()
        if reduction not in ("mean", "sum"):
            raise NotImplementedError("PerceptualLoss on MI355X supports reduction 'mean' and 'sum'")
        self.use_mse = use_mse
        self.reduction = reduction
        self._weights = weights
        self._stacks = {}
        _vgg.resolve_precision(precision)  # validates
        self.precision = precision

    def stack(self, device, dt: Optional[int] = None) -> "_vgg.VGGStack":
        """The trunk for `device` at C-ABI dtype `dt` (None: this module's precision)."""
        if dt is None:
            dt = _vgg.resolve_precision(self.precision)
        key = (str(device), dt)
        if key not in self._stacks:
            self._stacks[key] = _vgg.VGGStack(_vgg.VGG19_CFG, 36, device, self._weights, dtype=dt)
        return self._stacks[key]

    def forward(self, generated_img, target_img):
        if target_img.device != generated_img.device:
            target_img = target_img.to(generated_img.device)
        return _PerceptualFn.apply(generated_img, target_img, self, _vgg.resolve_precision(self.precision))

    def value_and_grad(self, gen, tgt, up: torch.Tensor, out: torch.Tensor, dt: Optional[int] = None) -> torch.Tensor:
        """Autograd-free form for the fused trainer (no host sync, HIP-graph capturable): writes the loss into
        out[0] and returns up[0] * d loss / d gen (NCHW fp32).  `dt`: trunk dtype override (None: `precision`)."""
        stack = self.stack(gen.device, dt)
        ft, _, _ = stack.forward(_vgg.prep_input(tgt, dtype=stack.dtype), save=False)
        fg, tape, _ = stack.forward(_vgg.prep_input(gen, dtype=stack.dtype), save=True)
        n = fg.numel()
        mode = 0 if self.use_mse else 1
        scale = 1.0 / n if self.reduction == "mean" else 1.0
        ws = torch.empty(query("feat_dist_workspace_doubles", n), dtype=torch.float64, device=gen.device)
        call("feat_dist_fwd", fg, ft, n, mode, scale, ws, out, stack.dtype)
        d = torch.empty_like(fg)
        call("feat_dist_bwd", fg, ft, n, mode, float(scale), 1, up, d, stack.dtype)
        return _vgg.input_grad(stack.backward(tape, d), gen)


class HybridLoss(nn.Module):
    """losses.py:72-89: total = l1 * L1 + lp * Perc; returns (total, l1, perc)."""

    def __init__(self, lambda_l1=1.0, lambda_perceptual=0.1, device="cuda"):
        super().__init__()
        self.device = _resolve_device(device)
        self.lambda_l1 = lambda_l1
        self.lambda_perceptual = lambda_perceptual
        self.perceptual_loss = PerceptualLoss(device=self.device)

    def forward(self, generated_img, target_img):
        l1_val = l1_loss(generated_img, target_img)
        if self.lambda_perceptual:
            perceptual_val = self.perceptual_loss(generated_img, target_img)
        else:
            perceptual_val = torch.zeros((), device=generated_img.device)
        total = self.lambda_l1 * l1_val + self.lambda_perceptual * perceptual_val
        return total, l1_val, perceptual_val


class _DeltaE00Fn(torch.autograd.Function):
    """mean CIEDE2000 (loss form) of rgb_to_lab(clamp01 gen) vs rgb_to_lab(clamp01 tgt); d/d gen by forward-mode AD
    in the kernel (color.hip)."""

    @staticmethod
    def forward(ctx, gen, tgt, eps):
        _lib.require_cuda(gen, tgt)
        if gen.shape != tgt.shape or gen.dim() != 4 or gen.shape[1] != 3:
            raise ValueError("DeltaE00Loss expects two [N,3,H,W] sRGB tensors of the same shape")
        gen = gen.detach().float().contiguous()
        tgt = tgt.detach().float().contiguous()
        N, _, H, W = gen.shape
        ws = torch.empty(query("de00_workspace_doubles", N * H * W), dtype=torch.float64, device=gen.device)
        out = torch.empty((), device=gen.device)
        call("de00_loss_fwd", gen, tgt, N, H, W, 1, float(eps), ws, out)
        ctx.save_for_backward(gen, tgt)
        ctx.eps = float(eps)
        return out

    @staticmethod
    def backward(ctx, up):
        gen, tgt = ctx.saved_tensors
        N, _, H, W = gen.shape
        up = up.float().contiguous().view(1)
        g = gt = None
        if ctx.needs_input_grad[0]:
            g = torch.empty_like(gen)
            call("de00_loss_bwd", gen, tgt, N, H, W, 1, ctx.eps, up, g)
        if ctx.needs_input_grad[1]:  # the loss is symmetric in (gen, tgt): the same kernel with the two swapped
            gt = torch.empty_like(tgt)
            call("de00_loss_bwd", tgt, gen, N, H, W, 1, ctx.eps, up, gt)
        return g, gt, None


class _CIEDE2000LabFn(torch.autograd.Function):
    """DeltaE00Loss._ciede2000 on Lab tensors [N,3,H,W] -> dE [N,H,W] (losses.py:98-136), both gradients by forward-mode
    AD per pixel (nbp_de00_lab_bwd; the form is symmetric, so d/dLab2 swaps the inputs)."""

    @staticmethod
    def forward(ctx, lab1, lab2, eps):
        _lib.require_cuda(lab1, lab2)
        if lab1.shape != lab2.shape or lab1.dim() != 4 or lab1.shape[1] != 3:
            raise ValueError("_ciede2000 expects two [N,3,H,W] Lab tensors of the same shape")
        lab1, lab2 = lab1.detach().contiguous(), lab2.detach().contiguous()
        N, _, H, W = lab1.shape
        out = torch.empty(N, H, W, device=lab1.device)
        call("de00_lab", lab1, lab2, N, H, W, 0, 1.0, 1.0, 1.0, float(eps), out)
        ctx.save_for_backward(lab1, lab2)
        ctx.eps = float(eps)
        return out

    @staticmethod
    def backward(ctx, g):
        lab1, lab2 = ctx.saved_tensors
        N, _, H, W = lab1.shape
        g = g.float().contiguous()
        d1 = d2 = None
        if ctx.needs_input_grad[0]:
            d1 = torch.empty_like(lab1)
            call("de00_lab_bwd", lab1, lab2, N, H, W, ctx.eps, g, d1)
        if ctx.needs_input_grad[1]:
            d2 = torch.empty_like(lab2)
            call("de00_lab_bwd", lab2, lab1, N, H, W, ctx.eps, g, d2)
        return d1, d2, None


class DeltaE00Loss(nn.Module):
    """losses.py:92-143 — mean ΔE00 (the reference's loss-form _ciede2000, eps 1e-6) between kornia-0.6.12
    rgb_to_lab(gen.clamp(0,1)) and rgb_to_lab(tgt.clamp(0,1)); one HIP kernel per direction (color.hip)."""

    def __init__(self, eps: float = 1e-6):
        super().__init__()
        self.eps = eps

    @staticmethod
    def _ciede2000(Lab1: torch.Tensor, Lab2: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
        """losses.py:98-136: the per-pixel loss-form CIEDE2000 of Lab [N,3,H,W] pairs -> [N,H,W] (differentiable in
        both arguments); one HIP kernel each way (color.hip)."""
        return _CIEDE2000LabFn.apply(Lab1.float(), Lab2.to(Lab1.device).float(), float(eps))

    def forward(self, gen_srgb01, tgt_srgb01):
        return _DeltaE00Fn.apply(gen_srgb01, tgt_srgb01, self.eps)


class SSIMLoss(nn.Module):
    """losses.py:146-155: kornia SSIMLoss(window_size=11, max_val=1, reduction) on clamp(0,1) inputs; reduction
    'mean' / 'sum' -> a scalar, 'none' -> the [N,C,H,W] loss map (kornia 0.6.12 ssim_loss); gradients to both
    inputs."""

    def __init__(self, window_size: int = 11, max_val: float = 1.0, reduction: str = "mean"):
        super().__init__()
        if window_size != 11:
            raise NotImplementedError("SSIMLoss on MI355X implements window_size=11 (the reference's only use)")
        if reduction not in _SSIM_REDUCTION:
            raise ValueError(f"Invalid reduction mode: {reduction}")  # kornia's ssim_loss message
        self.window_size = window_size
        self.max_val = max_val
        self.reduction = reduction

    def forward(self, gen_srgb01, tgt_srgb01):
        return _SSIMLossFn.apply(gen_srgb01, tgt_srgb01, self.window_size, self.max_val, 1, self.reduction)


class _PhysFullFn(torch.autograd.Function):
    """groups == 1 physics L1: conv2d(ReplicationPad(bhat), k [Co,C,kh,kw]) vs clamp?(a * ratio) under F.l1_loss's
    channel broadcast (nbp_phys_full_*)."""

    @staticmethod
    def forward(ctx, bhat, a, ratio_arr, ratio_full, k, clamp_align):
        _lib.require_cuda(bhat, a, k)
        bhat, a, kk = bhat.contiguous(), a.contiguous(), k.detach().contiguous()
        N, C, H, W = bhat.shape
        Co, Ca = kk.shape[0], a.shape[1]
        Cb = max(Co, Ca)
        ws = torch.empty(query("phys_l1_workspace_doubles", N, Cb, H, W), dtype=torch.float64, device=bhat.device)
        loss = torch.empty((), device=bhat.device)
        want = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        sign = torch.empty(N, Cb, H, W, device=bhat.device) if want else None
        call("phys_full_fwd", bhat, a, ratio_arr, ratio_full, kk, N, C, Co, Ca, H, W, kk.shape[-2], kk.shape[-1],
             clamp_align, ws, loss, sign)
        ctx.save_for_backward(sign, kk, a, ratio_arr)
        ctx.dims = (N, C, Co, Ca, H, W)
        ctx.args = (clamp_align, ratio_full)
        return loss

    @staticmethod
    def backward(ctx, up):
        sign, kk, a, ratio_arr = ctx.saved_tensors
        N, C, Co, Ca, H, W = ctx.dims
        clamp_align, ratio_full = ctx.args
        up = up.float().contiguous().view(1)
        g = ga = None
        if ctx.needs_input_grad[0]:
            g = torch.empty(N, C, H, W, device=sign.device)
            call("phys_full_bwd", sign, kk, up, N, C, Co, Ca, H, W, kk.shape[-2], kk.shape[-1], g)
        if ctx.needs_input_grad[1]:
            ga = torch.empty_like(a)
            call("phys_a_bwd", sign, a, ratio_arr, ratio_full, N, Ca, max(Co, Ca), H, W, 0, clamp_align, up, ga)
        return g, ga, None, None, None, None


class PhysicsConsistencyLoss(nn.Module):
    """losses.py:158-192: |K * ReplicationPad(Bhat_raw) - clamp(A_raw * ratio)|_1 with the UN-normalised K.
    The reference's kernel forms, with its groups logic (:182-190): a shared [1,1,kh,kw] kernel is broadcast to every
    channel and a [C,1,kh,kw] one is applied per channel (depthwise, nbp_phys_l1_*); any other [Co,1,kh,kw] kernel is
    expanded to [Co,C,kh,kw] and a full [Co,C,kh,kw] kernel used as is (groups = 1, nbp_phys_full_*), the L1 taken over
    F.l1_loss's broadcast of [N,Co,H,W] against A's channels.  Kernel / channel combinations the reference's conv2d
    rejects raise RuntimeError as there."""

    def __init__(self, K_kernel: torch.Tensor, device: str = "cuda", clamp_align: bool = True):
        super().__init__()
        if K_kernel is None:
            raise ValueError("K_kernel must be provided for PhysicsConsistencyLoss")
        self.register_buffer("K", K_kernel.to(device))
        self.K: torch.Tensor
        self.clamp_align = clamp_align

    def forward(self, Bhat_raw, A_raw, expo_ratio):
        if expo_ratio.dim() == 1:
            expo_ratio = expo_ratio.view(-1, 1, 1, 1)
        C = Bhat_raw.shape[1]
        k = self.K
        kh, kw = k.shape[-2:]
        if k.shape[0] == 1 and C > 1:  # shared kernel broadcast to every channel (:184-185)
            if k.shape[1] != 1:
                raise RuntimeError(f"PhysicsConsistencyLoss: kernel {tuple(k.shape)} cannot be expanded to "
                                   f"{(C, 1, kh, kw)}")
            k = k.expand(C, 1, kh, kw)
        groups = C if k.shape[0] == C else 1  # :187
        if groups == 1 and k.shape[1] == 1 and C != 1:  # :189-190
            k = k.expand(k.shape[0], C, kh, kw)
        if k.shape[1] != C // groups:  # what F.conv2d rejects
            raise RuntimeError(f"PhysicsConsistencyLoss: conv2d weight {tuple(k.shape)} with groups={groups} does not "
                               f"match {C} input channels")
        if groups == C and k.shape[0] == C and k.shape[1] == 1:  # depthwise (per-channel, or the broadcast shared one)
            r, full = _ratio_array(expo_ratio, A_raw)
            shared = int(self.K.shape[0] == 1 and C > 1)
            kd = self.K if shared else k
            return _PhysL1Fn.apply(Bhat_raw, A_raw, r, full, kd.to(Bhat_raw.dtype), shared, 1, 0, 0,
                                   int(self.clamp_align))
        Co, Ca = k.shape[0], A_raw.shape[1]
        if A_raw.shape[0] != Bhat_raw.shape[0] or A_raw.shape[2:] != Bhat_raw.shape[2:] or not (
                Co == Ca or Co == 1 or Ca == 1):
            raise RuntimeError(f"PhysicsConsistencyLoss: conv output {(Bhat_raw.shape[0], Co, *Bhat_raw.shape[2:])} "
                               f"does not broadcast with A {tuple(A_raw.shape)}")
        if Co != Ca:  # F.l1_loss warns on a broadcast target (torch.nn.functional.l1_loss)
            warnings.warn(f"Using a target size ({torch.Size([A_raw.shape[0], Ca, *A_raw.shape[2:]])}) that is "
                          f"different to the input size ({torch.Size([Bhat_raw.shape[0], Co, *Bhat_raw.shape[2:]])}). "
                          "This will likely lead to incorrect results due to broadcasting. Please ensure they have "
                          "the same size.", UserWarning)
        r, full = _ratio_array(expo_ratio, A_raw)
        return _PhysFullFn.apply(Bhat_raw, A_raw.float(), r, full, k.float().contiguous(), int(self.clamp_align))


def align_exposure_srgb(a_srgb: torch.Tensor, ratio) -> torch.Tensor:
    """losses.py:195-203: clamp(a * ratio, 0, 1)."""
    _lib.require_cuda(a_srgb)
    a = a_srgb.contiguous()
    N, C, H, W = a.shape
    r, full = _ratio_array(ratio, a)
    out = torch.empty_like(a)
    call("align_exposure", a, r, full, out, N, C, H * W)
    return out


class PhysicalConsistencyLossSRGB(nn.Module):
    """losses.py:206-220: L1(PSF(bhat_srgb), align(a_srgb; ratio)) — one fused kernel, adjoint backward."""

    def __init__(self, psf_module: nn.Module):
        super().__init__()
        self.psf = psf_module

    def forward(self, bhat_srgb, a_srgb, ratio, _clamp_bhat: bool = False, _clamp_a: bool = False):
        if bhat_srgb.shape[1] != 3:
            raise AssertionError("CrosstalkPSF expects sRGB inputs (3 channels).")
        k = self.psf.kernel
        mono = getattr(self.psf, "mode", "rgb") == "mono"
        r, full = _ratio_array(ratio, a_srgb)
        return _PhysL1Fn.apply(bhat_srgb, a_srgb, r, full, k.to(bhat_srgb.dtype), int(mono), 0, int(_clamp_bhat),
                               int(_clamp_a), 1)


class HybridLossPlus(nn.Module):
    """losses.py:223-372: weighted sum of L1_raw, Perc, LPIPS, DeltaE, SSIM, Phys in that order; returns
    (L_total, logs).  `check_finite=True` keeps the reference's per-term host-side finiteness check
    (losses.py:298-306, a host sync per term); the fused trainer turns it off and checks once per log step."""

    def __init__(self, device: str = "cuda", w_l1_raw: float = 1.0, w_perc: float = 0.02, w_lpips: float = 0.0,
                 w_deltaE: float = 0.02, w_ssim: float = 0.05, w_phys: float = 0.10, use_deltaE: bool = True,
                 use_ssim: bool = True, use_lpips: bool = False, use_phys: bool = True, use_uncertainty: bool = False,
                 physics_kernel: Optional[torch.Tensor] = None, physics_psf_module: Optional[nn.Module] = None):
        super().__init__()
        device = _resolve_device(device)
        self.register_buffer("_zero", torch.tensor(0.0), persistent=False)
        self.perc = PerceptualLoss(device=device)
        self.deltaE = DeltaE00Loss() if use_deltaE else None
        self.ssim = SSIMLoss() if use_ssim else None
        self.lpips = LPIPS(net="vgg") if use_lpips else None  # lpips.LPIPS(net='vgg') restated (lpips.py)
        self.phys = PhysicsConsistencyLoss(physics_kernel, device=device) if use_phys and physics_kernel is not None else None
        self.phys_srgb = PhysicalConsistencyLossSRGB(physics_psf_module.to(device)) if (
            use_phys and physics_psf_module is not None) else None
        self.use_uncertainty = use_uncertainty
        if use_uncertainty:
            self.log_sigma = nn.ParameterDict({k: nn.Parameter(torch.zeros(())) for k in
                                               ("l1", "perc", "lpips", "de", "ssim", "phys")})
        else:
            self.w = dict(l1=w_l1_raw, perc=w_perc, lpips=w_lpips, de=w_deltaE, ssim=w_ssim, phys=w_phys)
        self.check_finite = True

    def _ensure_finite(self, name: str, value: torch.Tensor):
        if not self.check_finite:
            return
        if not torch.isfinite(value).all():
            raise RuntimeError(f"HybridLossPlus detected non-finite values in term '{name}'.")

    def _weighted(self, name, val):
        if val is None:
            z = self._zero.clone()
            return z, z.detach()
        if self.use_uncertainty:
            s = self.log_sigma[name]
            return val * torch.exp(-2 * s) + s, val.detach()
        return self.w[name] * val, val.detach()

    def _active(self, name):
        return self.use_uncertainty or self.w[name] != 0

    def _term(self, name, fn):
        """A term the reference always evaluates: with weight 0 its value is still logged, but it is computed without
        building a backward (0 * term contributes a zero gradient)."""
        if self._active(name):
            return fn()
        with torch.no_grad():
            return fn()

    def forward(self, *, Bhat_raw, B_raw, A_raw, expo_ratio, Bhat_srgb01, B_srgb01, A_srgb01=None):
        logs: Dict[str, torch.Tensor] = {}
        L_total = 0.0
        L_l1 = l1_loss(Bhat_raw, B_raw)
        self._ensure_finite("L1_raw", L_l1)
        Lw, logs["L1_raw"] = self._weighted("l1", L_l1)
        L_total = L_total + Lw
        L_p = self._term("perc", lambda: self.perc(Bhat_srgb01, B_srgb01))  # always evaluated (losses.py:337)
        self._ensure_finite("Perc", L_p)
        Lw, logs["Perc"] = self._weighted("perc", L_p)
        L_total = L_total + Lw
        if self.lpips is not None:
            L_lp = self.lpips(Bhat_srgb01, B_srgb01).mean()
            self._ensure_finite("LPIPS", L_lp)
            Lw, logs["LPIPS"] = self._weighted("lpips", L_lp)
            L_total = L_total + Lw
        if self.deltaE is not None:
            L_de = self._term("de", lambda: self.deltaE(Bhat_srgb01, B_srgb01))
            self._ensure_finite("DeltaE", L_de)
            Lw, logs["DeltaE"] = self._weighted("de", L_de)
            L_total = L_total + Lw
        if self.ssim is not None:
            L_ss = self.ssim(Bhat_srgb01, B_srgb01)
            self._ensure_finite("SSIM", L_ss)
            Lw, logs["SSIM"] = self._weighted("ssim", L_ss)
            L_total = L_total + Lw
        if self.phys is not None:
            L_ph = self.phys(Bhat_raw, A_raw, expo_ratio)
            self._ensure_finite("Phys_raw", L_ph)
            Lw, logs["Phys"] = self._weighted("phys", L_ph)
            L_total = L_total + Lw
        elif self.phys_srgb is not None and A_srgb01 is not None:
            L_phs = self.phys_srgb(Bhat_srgb01, A_srgb01, expo_ratio)
            self._ensure_finite("Phys_srgb", L_phs)
            Lw, logs["Phys"] = self._weighted("phys", L_phs)
            L_total = L_total + Lw
        logs["Total"] = L_total.detach()
        return L_total, logs
