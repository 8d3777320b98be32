"""VGG feature stacks on MI355X for the perceptual and LPIPS (row 22) terms.

A frozen VGG `features` prefix (3x3 conv + ReLU, 2x2 max pool) runs over NHWC bf16 activations:
  * every conv is an implicit GEMM on the bf16 MFMA kernel (nbp_conv3x3_bf16: the 3x3 neighbourhood gathered in the
    A-tile loader, K = 9*Cin), bias + ReLU fused in the epilogue;
  * the input gradient (weights are frozen: no weight gradients) is the same implicit GEMM over the gradient map with
    the tap-flipped, transposed weights; the ReLU masks ride in the epilogue (conv -> conv) or in the pool backward
    (conv -> pool -> conv); max pools keep their argmax.
Storage / operand type `dtype`: 0 fp32 (the reference's own trunk: PerceptualLoss feeds `x.float()` to the conv stack,
NewBP_model/losses.py:63-69; implicit GEMM on the fp32 MFMA, exact products), 1 bf16 or 2 fp16 (16-bit MFMA operands,
fp32 accumulation; fp16 is the reference's autocast dtype, used under the trainer's dynamic loss scaling -- its 11-bit
significand keeps the deep input gradient far closer to fp32).

Pretrained ImageNet weights (torchvision / lpips downloads) are not available offline: `weights=None` builds the
architecture with a deterministic synthetic initialisation (kaiming-normal fan-out as torchvision, seed 0); pass a
state_dict or a checkpoint path (loaded with torch.load(weights_only=True)) to use real weights.
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Optional, Sequence, Union

import torch

from . import _lib
from ._lib import call

# torchvision VGG configurations ('M' = max pool)
VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _layers(cfg, n_modules: int):
    """[(kind, torch features index, cin, cout)] for features[:n_modules] (conv and relu are separate modules)."""
    out, idx, cin = [], 0, 3
    for v in cfg:
        if idx >= n_modules:
            break
        if v == "M":
            out.append(("pool", idx, cin, cin))
            idx += 1
        else:
            out.append(("conv", idx, cin, v))  # conv at idx, its ReLU at idx + 1
            idx += 2
            cin = v
    return out


def synthetic_state_dict(cfg, n_modules: int, seed: int = 0) -> Dict[str, torch.Tensor]:
    """torchvision's VGG init (kaiming_normal_(fan_out, relu), zero bias) from a fixed generator."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for kind, idx, cin, cout in _layers(cfg, n_modules):
        if kind == "conv":
            std = (2.0 / (cout * 9)) ** 0.5
            sd[f"{idx}.weight"] = torch.randn(cout, cin, 3, 3, generator=g) * std
            sd[f"{idx}.bias"] = torch.zeros(cout)
    return sd


def _pad8(c: int) -> int:
    return (c + 7) // 8 * 8


TORCH_DTYPE = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}
PRECISIONS = {"fp32": 0, "bf16": 1, "fp16": 2}


def resolve_precision(precision: str) -> int:
    """C-ABI dtype of a trunk precision.  "auto" follows torch.autocast as the reference's fp32 module does under
    it (fp16 / bf16 conv operands inside an enabled CUDA autocast region, fp32 otherwise)."""
    if precision == "auto":
        if torch.is_autocast_enabled("cuda"):
            return 2 if torch.get_autocast_dtype("cuda") == torch.float16 else 1
        return 0
    if precision not in PRECISIONS:
        raise ValueError(f"VGG trunk precision must be 'auto', 'fp32', 'bf16' or 'fp16', got {precision!r}")
    return PRECISIONS[precision]


class VGGStack:
    """Frozen VGG features[:n_modules] on device.  forward() returns the final post-ReLU map (NHWC bf16) and,
    when asked, the post-ReLU maps at `taps` (torch module indices of ReLUs); backward() maps d(final pre-ReLU map)
    plus optional tap gradients to d(prepared input) [B][H][W][8] fp32."""

    def __init__(self, cfg, n_modules: int, device, weights: Union[None, str, Dict[str, torch.Tensor]] = None,
                 seed: int = 0, dtype: int = 1):
        if dtype not in (0, 1, 2):
            raise ValueError("VGGStack dtype: 0 (fp32), 1 (bf16) or 2 (fp16)")
        self.cfg, self.n_modules, self.device = cfg, n_modules, torch.device(device)
        self.dtype = dtype
        self.tdt = TORCH_DTYPE[dtype]
        self.ydt = 0 if dtype == 0 else 1  # nbp_conv3x3_bf16's y_dtype for an activation-typed output
        if weights is None:
            warnings.warn("VGG: ImageNet weights are not available offline; using a deterministic synthetic "
                          "initialisation (pass weights=<state_dict or path> for real weights)", RuntimeWarning)
            sd = synthetic_state_dict(cfg, n_modules, seed)
        elif isinstance(weights, str):
            sd = torch.load(weights, map_location="cpu", weights_only=True)
        else:
            sd = dict(weights)
        sd = {k[len("features."):] if k.startswith("features.") else k: v for k, v in sd.items()}
        self.layers = []
        for kind, idx, cin, cout in _layers(cfg, n_modules):
            if kind == "pool":
                self.layers.append(dict(kind="pool", idx=idx))
                continue
            w = sd[f"{idx}.weight"].float()
            b = sd[f"{idx}.bias"].float()
            if tuple(w.shape) != (cout, cin, 3, 3):
                raise ValueError(f"VGG layer {idx}: weight shape {tuple(w.shape)} != {(cout, cin, 3, 3)}")
            cp = _pad8(cin)
            wp = torch.zeros(cout, cp, 3, 3)
            wp[:, :cin] = w
            # forward operand [Cout][tap][Cin_pad]; input-gradient operand [Cin_pad][tap'][Cout], tap' = 8 - tap
            wf = wp.permute(0, 2, 3, 1).reshape(cout, 9, cp)
            wt = wf.flip(1).permute(2, 1, 0).contiguous()
            self.layers.append(dict(kind="conv", idx=idx, cin=cp, cout=cout,
                                    wf=wf.to(self.device, self.tdt).contiguous(),
                                    wt=wt.to(self.device, self.tdt).contiguous(),
                                    bias=b.to(self.device).contiguous()))

    # ------------------------------------------------------------------ forward
    def forward(self, x8: torch.Tensor, save: bool, taps: Sequence[int] = ()):
        """x8: [B][H][W][8] prepared input (prep_input with this stack's dtype).  Returns (final post-ReLU map, tape,
        {tap index: post map})."""
        B, H, W, _ = x8.shape
        h, w, feat = H, W, x8
        tape: List = []
        tapped = {}
        for L in self.layers:
            if L["kind"] == "conv":
                y = torch.empty(B, h, w, L["cout"], device=x8.device, dtype=self.tdt)
                call("conv3x3_bf16", feat, B, h, w, L["cin"], L["wf"], L["cout"], L["bias"], 0, None, y, self.ydt,
                     self.dtype)
                if save:
                    tape.append(("conv", L, (B, h, w), y))
                if L["idx"] + 1 in taps:
                    tapped[L["idx"] + 1] = y
                feat = y
            else:
                C = feat.shape[-1]
                ho, wo = h // 2, w // 2
                y = torch.empty(B, ho, wo, C, device=x8.device, dtype=self.tdt)
                idx = torch.empty(B, ho, wo, C, device=x8.device, dtype=torch.uint8)
                call("maxpool2_fwd", feat, B, h, w, C, y, idx, self.dtype)
                if save:
                    tape.append(("pool", (B, h, w, C), idx, feat))
                feat, h, w = y, ho, wo
        return feat, tape, tapped

    # ------------------------------------------------------------------ input gradient
    def backward(self, tape, d_last_pre: torch.Tensor, tap_grads: Optional[Dict[int, torch.Tensor]] = None):
        """d_last_pre: gradient w.r.t. the last conv's PRE-ReLU output (NHWC, the stack's type).  tap_grads: {relu index:
        gradient w.r.t. that post-ReLU map} added where the walk passes it.  Returns d(prepared input) fp32 [B,H,W,8]."""
        tap_grads = tap_grads or {}
        d = d_last_pre
        n = len(tape)
        for k in range(n - 1, -1, -1):
            rec = tape[k]
            if rec[0] != "conv":
                continue
            L, (B, h, w) = rec[1], rec[2]
            prev = tape[k - 1] if k > 0 else None
            if prev is None:  # first conv: gradient of the prepared input
                d8 = torch.empty(B, h, w, L["cin"], device=d.device)
                call("conv3x3_bf16", d, B, h, w, L["cout"], L["wt"], L["cin"], None, 1, None, d8, 0, self.dtype)
                return d8
            if prev[0] == "conv":  # conv -> ReLU -> conv: mask by the previous post map in the epilogue
                post = prev[3]
                dn = torch.empty(B, h, w, L["cin"], device=d.device, dtype=self.tdt)
                call("conv3x3_bf16", d, B, h, w, L["cout"], L["wt"], L["cin"], None, 2, post, dn, self.ydt, self.dtype)
                tg = tap_grads.get(prev[1]["idx"] + 1)
                if tg is not None:  # + d(tap) * relu mask
                    call("add_relu_masked", dn, tg.to(self.tdt).contiguous(), post, dn.numel(), self.dtype)
                d = dn
            else:  # conv -> ReLU -> pool -> conv
                (_, (Bp, hp, wp, C), idx, pool_in) = prev
                dp = torch.empty(B, h, w, L["cin"], device=d.device, dtype=self.tdt)
                call("conv3x3_bf16", d, B, h, w, L["cout"], L["wt"], L["cin"], None, 1, None, dp, self.ydt, self.dtype)
                dn = torch.empty(Bp, hp, wp, C, device=d.device, dtype=self.tdt)
                call("maxpool2_bwd", dp, idx, pool_in, Bp, hp, wp, C, dn, self.dtype)
                conv_before = tape[k - 2]
                tg = tap_grads.get(conv_before[1]["idx"] + 1)
                if tg is not None:
                    call("add_relu_masked", dn, tg.to(self.tdt).contiguous(), pool_in, dn.numel(), self.dtype)
                d = dn
        raise RuntimeError("VGG backward: tape has no conv layer")


def prep_input(x: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD, clamp: bool = True, dtype: int = 1) -> torch.Tensor:
    """NCHW fp32 [B,3,H,W] -> NHWC [B,H,W,8] (the stack's type) of (clamp01(x) - mean) / std (nbp_vgg_prep)."""
    _lib.require_cuda(x)
    if x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"VGG input must be [B,3,H,W], got {tuple(x.shape)}")
    x = x.float().contiguous()
    B, _, H, W = x.shape
    y = torch.empty(B, H, W, 8, device=x.device, dtype=TORCH_DTYPE[dtype])
    call("vgg_prep", x, B, H, W, int(clamp), *[float(v) for v in mean], *[float(v) for v in std], y, dtype)
    return y


def input_grad(d8: torch.Tensor, x: torch.Tensor, std=IMAGENET_STD, clamp: bool = True) -> torch.Tensor:
    """d(prepared input) [B,H,W,8] fp32 -> d x NCHW fp32 (nbp_vgg_input_grad)."""
    B, _, H, W = x.shape
    dx = torch.empty(B, 3, H, W, device=x.device)
    call("vgg_input_grad", d8, x.float().contiguous(), B, H, W, int(clamp), *[float(v) for v in std], dx)
    return dx
