"""LPIPS (lpips==0.1.4, `lpips.LPIPS(net='vgg' | 'alex')`) on MI355X — the HybridLossPlus LPIPS term (net='vgg',
NewBP_model/losses.py:265-274, 342-346) and the validation metric's default backbone (net='alex',
metrics/lpips_metric.py:43-57, basicsr/metrics/lowlight_metrics.py:223-226).

Restated from the package's published algorithm (the package and its weights are absent here: parity unpinned):
ScalingLayer (x - shift) / scale with shift (-.030, -.088, -.188), scale (.458, .448, .450) (inputs taken as [-1, 1];
`normalize=True` maps [0, 1] first); VGG16 features with taps relu1_2, relu2_2, relu3_3, relu4_3, relu5_3; per tap
normalize_tensor over channels, squared difference, the non-negative 1x1 'lin' head, spatial average; sum over taps.
Output [N, 1, 1, 1] per image like lpips.  The VGG16 trunk is the implicit-GEMM MFMA stack of vgg.py (fp32 like the
package's own module, or 16-bit operands: `precision`); the tap distances and their gradients are nbp_lpips_tap_*
kernels; the tap gradients join the VGG backward walk.

net='alex' (torchvision alexnet.features taps relu1..relu5: conv 11x11/4 pad 2 -> pool 3/2 -> conv 5x5 pad 2 -> pool 3/2 ->
3 x conv 3x3 pad 1) runs its strided convs as implicit GEMMs on the MFMA kernels (nbp_conv2d_16) with 3x3/2 max pools
(nbp_maxpool_k_fwd, argmax kept); its input gradient (BASELINE.json cfg3 names LPIPS(alex) in the training loss) runs
the stride-1 convs' transposes as implicit GEMMs with the ReLU mask in the epilogue, the overlapping pools through
their argmax (nbp_maxpool_k_bwd) and the 11x11/4 first conv as a direct transposed conv (nbp_alex_conv0_input_grad).

Weights: pretrained VGG16 / AlexNet + 'lin' weights cannot be downloaded here.  `weights` takes an lpips-style state_dict
(`net.sliceK.N.*`, `linK.model.1.weight`) or a path (torch.load(weights_only=True)); None gives a deterministic
synthetic model (kaiming VGG16, lin = |N(0, 0.1)|, seed 0).
"""
from __future__ import annotations

import re
import warnings
from typing import Dict, Optional

import torch
import torch.nn as nn

from . import _lib
from . import vgg as _vgg
from ._lib import call, query

SHIFT = (-0.030, -0.088, -0.188)
SCALE = (0.458, 0.448, 0.450)
TAPS = (3, 8, 15, 22, 29)        # relu1_2, relu2_2, relu3_3, relu4_3, relu5_3 in vgg16.features
TAP_CH = (64, 128, 256, 512, 512)
# torchvision alexnet.features: (module index, cin, cout, kernel, stride, pad) convs, max pools 3/2 at 2 and 5
ALEX_CONVS = ((0, 3, 64, 11, 4, 2), (3, 64, 192, 5, 1, 2), (6, 192, 384, 3, 1, 1), (8, 384, 256, 3, 1, 1),
              (10, 256, 256, 3, 1, 1))
ALEX_TAP_CH = (64, 192, 384, 256, 256)  # relu1 .. relu5 (module indices 1, 4, 7, 9, 11)


def alex_synthetic_state_dict(seed: int = 0) -> Dict[str, torch.Tensor]:
    """torch's default Conv2d init (kaiming-uniform a = sqrt(5): U(+-1/sqrt(fan_in)) weights and biases) from a fixed
    generator -- torchvision's AlexNet keeps the default init."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for idx, cin, cout, k, _, _ in ALEX_CONVS:
        bound = 1.0 / (cin * k * k) ** 0.5
        sd[f"{idx}.weight"] = (torch.rand(cout, cin, k, k, generator=g) * 2 - 1) * bound
        sd[f"{idx}.bias"] = (torch.rand(cout, generator=g) * 2 - 1) * bound
    return sd


class AlexStack:
    """Frozen alexnet.features[:12] on device: taps() returns the five post-ReLU maps (NHWC, the stack's type) and,
    with save=True, a tape for backward(): the input gradient from the tap gradients (stride-1 convs as implicit-GEMM
    convs with tap-flipped weights and the ReLU mask in the epilogue, overlapping 3x3/2 max pools through their argmax,
    the 11x11/4 first conv as a direct transposed conv)."""

    def __init__(self, device, feats: Dict[str, torch.Tensor], dtype: int = 1):
        self.device, self.dtype = torch.device(device), dtype
        self.tdt = _vgg.TORCH_DTYPE[dtype]
        self.convs = []
        for i, (idx, cin, cout, k, st, pad) in enumerate(ALEX_CONVS):
            w = feats[f"{idx}.weight"].float()
            if tuple(w.shape) != (cout, cin, k, k):
                raise ValueError(f"alexnet layer {idx}: weight shape {tuple(w.shape)} != {(cout, cin, k, k)}")
            cp = _vgg._pad8(cin)
            wp = torch.zeros(cout, cp, k, k)
            wp[:, :cin] = w
            wf = wp.permute(0, 2, 3, 1).reshape(cout, k * k, cp)
            L = dict(w=wf.to(self.device, self.tdt).contiguous(),
                     b=feats[f"{idx}.bias"].float().to(self.device).contiguous(), cin=cp, cout=cout, k=k, st=st, pad=pad)
            if i == 0:  # [Cout][121][8] fp32 for the direct transposed conv
                L["wd"] = wf.to(self.device).contiguous()
            else:  # stride 1, 'same' padding: the input gradient is the conv with W'[c][t'][n] = W[n][k*k-1-t'][c]
                L["wt"] = wf.flip(1).permute(2, 1, 0).to(self.device, self.tdt).contiguous()
            self.convs.append(L)

    def taps(self, x8: torch.Tensor, save: bool = False):
        B, H, W, _ = x8.shape
        feat, h, w, out = x8, H, W, []
        tape = []
        for i, L in enumerate(self.convs):
            if i in (1, 2):  # MaxPool2d(3, 2) before conv 2 and conv 3
                ho, wo = (h - 3) // 2 + 1, (w - 3) // 2 + 1
                y = torch.empty(B, ho, wo, feat.shape[-1], device=x8.device, dtype=self.tdt)
                idx = torch.empty(B, ho, wo, feat.shape[-1], device=x8.device, dtype=torch.uint8) if save else None
                call("maxpool_k_fwd", feat, B, h, w, feat.shape[-1], 3, 2, y, idx, self.dtype)
                if save:
                    tape.append(("pool", (B, h, w, feat.shape[-1]), idx, feat))
                feat, h, w = y, ho, wo
            ho, wo = (h + 2 * L["pad"] - L["k"]) // L["st"] + 1, (w + 2 * L["pad"] - L["k"]) // L["st"] + 1
            y = torch.empty(B, ho, wo, L["cout"], device=x8.device, dtype=self.tdt)
            call("conv2d_16", feat, B, h, w, L["cin"], L["w"], L["cout"], L["k"], L["k"], L["st"], L["pad"], L["b"], 0,
                 None, y, self.dtype)
            if save:
                tape.append(("conv", i, (B, h, w, ho, wo), y))
            out.append(y)
            feat, h, w = y, ho, wo
        return (out, tape) if save else out

    def backward(self, tape, tap_grads) -> torch.Tensor:
        """tap_grads[k]: gradient w.r.t. tap k's post-ReLU map (k = 0..4).  Returns d(prepared input) [B,H,W,8] fp32."""
        last = tape[-1][3]
        d = torch.zeros_like(last)  # pre-ReLU gradient of the last conv
        call("add_relu_masked", d, tap_grads[4].to(self.tdt).contiguous(), last, d.numel(), self.dtype)
        for t in range(len(tape) - 1, -1, -1):
            rec = tape[t]
            if rec[0] != "conv":
                continue
            i, (B, h, w, ho, wo) = rec[1], rec[2]
            L = self.convs[i]
            if i == 0:
                d8 = torch.empty(B, h, w, 8, device=d.device)
                call("alex_conv0_input_grad", d, L["wd"], B, h, w, ho, wo, L["cout"], d8, self.dtype)
                return d8
            prev = tape[t - 1]
            if prev[0] == "conv":  # conv -> ReLU -> conv: mask by the previous post map in the epilogue
                post = prev[3]
                dn = torch.empty(B, h, w, L["cin"], device=d.device, dtype=self.tdt)
                call("conv2d_16", d, B, h, w, L["cout"], L["wt"], L["cin"], L["k"], L["k"], 1, L["pad"], None, 2, post,
                     dn, self.dtype)
                call("add_relu_masked", dn, tap_grads[i - 1].to(self.tdt).contiguous(), post, dn.numel(), self.dtype)
                d = dn
            else:  # conv -> ReLU -> pool(3, 2) -> conv
                (_, (Bp, hp, wp, C), idx, pool_in) = prev
                dp = torch.empty(B, h, w, L["cin"], device=d.device, dtype=self.tdt)
                call("conv2d_16", d, B, h, w, L["cout"], L["wt"], L["cin"], L["k"], L["k"], 1, L["pad"], None, 1, None,
                     dp, self.dtype)
                dn = torch.empty(Bp, hp, wp, C, device=d.device, dtype=self.tdt)
                call("maxpool_k_bwd", dp, idx, pool_in, Bp, hp, wp, C, 3, 2, dn, self.dtype)
                call("add_relu_masked", dn, tap_grads[i - 1].to(self.tdt).contiguous(), pool_in, dn.numel(), self.dtype)
                d = dn
        raise RuntimeError("alex backward: tape has no first conv")


def _split_state_dict(sd: Dict[str, torch.Tensor]):
    feats, lins = {}, {}
    for k, v in sd.items():
        m = re.match(r"(?:net\.)?slice\d\.(\d+)\.(weight|bias)$", k)
        if m:
            feats[f"{m.group(1)}.{m.group(2)}"] = v
            continue
        m = re.match(r"lin(\d)\.model\.1\.weight$", k)
        if m:
            lins[int(m.group(1))] = v.reshape(-1).float()
    return feats, lins


def _trunk_taps(stack, x, save):
    """Prepared input -> (five tap maps, tape) for either backbone."""
    x8 = _vgg.prep_input(x, SHIFT, SCALE, clamp=False, dtype=stack.dtype)
    if isinstance(stack, AlexStack):
        return stack.taps(x8, save=True) if save else (stack.taps(x8), None)
    _, tape, t = stack.forward(x8, save=save, taps=TAPS)
    return [t[tap] for tap in TAPS], tape


def _trunk_backward(stack, tape, grads):
    """Tap gradients (list of 5) -> d(prepared input) [B,H,W,8] fp32 for either backbone."""
    if isinstance(stack, AlexStack):
        return stack.backward(tape, grads)
    last = tape[-1][3]  # relu5_3 is the VGG stack's last map: its pre-ReLU gradient
    d_last = torch.zeros_like(grads[-1])
    call("add_relu_masked", d_last, grads[-1], last, d_last.numel(), stack.dtype)
    return stack.backward(tape, d_last, tap_grads={tap: g for tap, g in zip(TAPS[:-1], grads[:-1])})


def _tap_distances(stack, lins, t0, t1, out, want_grad, up=None, accumulate_first=False):
    """out[n] (+)= sum_k lin_k-weighted distance of tap k; with want_grad the per-tap gradients w.r.t. t0."""
    N = t0[0].shape[0]
    grads = []
    for k in range(5):
        a, b = t0[k], t1[k]
        HW, C = a.shape[1] * a.shape[2], a.shape[3]
        ws = torch.empty(query("lpips_tap_workspace_doubles", N, HW), dtype=torch.float64, device=a.device)
        call("lpips_tap_fwd", a, b, lins[k], N, HW, C, int(k > 0 or accumulate_first), ws, out, stack.dtype)
        if want_grad:
            g = torch.empty_like(a)
            call("lpips_tap_bwd", a, b, lins[k], N, HW, C, up, g, stack.dtype)
            grads.append(g)
    return grads


class _LPIPSFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, in0, in1, module, normalize, dt):
        _lib.require_cuda(in0, in1)
        if in0.shape != in1.shape or in0.dim() != 4 or in0.shape[1] != 3:
            raise ValueError("LPIPS expects two [N,3,H,W] tensors of the same shape")
        x0 = in0.detach().float()
        x1 = in1.detach().float()
        if normalize:  # [0,1] -> [-1,1]
            x0, x1 = 2 * x0 - 1, 2 * x1 - 1
        stack, lins = module.parts(in0.device, dt)
        want0, want1 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        with torch.no_grad():
            # the ScalingLayer is the prologue's (x - mean) / std with mean = shift, std = scale (no clamp)
            t0, tape0 = _trunk_taps(stack, x0, want0)
            t1, tape1 = _trunk_taps(stack, x1, want1)
        N = in0.shape[0]
        out = torch.zeros(N, device=in0.device)
        _tap_distances(stack, lins, t0, t1, out, False)
        if want0 or want1:
            ctx.tapes, ctx.t0, ctx.t1, ctx.stack, ctx.lins = (tape0, tape1), t0, t1, stack, lins
            ctx.normalize = normalize
            ctx.save_for_backward(x0, x1)
        return out.view(N, 1, 1, 1)

    @staticmethod
    def backward(ctx, up):
        x0, x1 = ctx.saved_tensors
        up = up.float().contiguous().view(-1)
        outs = [None, None]
        # the tap distance sum_c w_c (a/|a| - b/|b|)^2 is symmetric: d/d in1 is the tap gradient with the maps swapped
        for side, (mine, other, x) in enumerate(((ctx.t0, ctx.t1, x0), (ctx.t1, ctx.t0, x1))):
            if not ctx.needs_input_grad[side]:
                continue
            grads = []
            for k in range(5):
                a, b = mine[k], other[k]
                g = torch.empty_like(a)
                call("lpips_tap_bwd", a, b, ctx.lins[k], a.shape[0], a.shape[1] * a.shape[2], a.shape[3], up, g,
                     ctx.stack.dtype)
                grads.append(g)
            d8 = _trunk_backward(ctx.stack, ctx.tapes[side], grads)
            dx = _vgg.input_grad(d8, x, SCALE, clamp=False)
            outs[side] = dx * 2 if ctx.normalize else dx
        ctx.tapes = ctx.t0 = ctx.t1 = None
        return outs[0], outs[1], None, None, None


class LPIPS(nn.Module):
    """lpips.LPIPS(net='vgg') drop-in: forward(in0, in1, retPerLayer=False, normalize=False) -> [N,1,1,1]."""

    def __init__(self, net: str = "vgg", weights=None, version: str = "0.1", precision: str = "auto", **_):
        super().__init__()
        if net not in ("vgg", "alex"):
            raise NotImplementedError("LPIPS on MI355X implements net='vgg' (the HybridLossPlus term) and net='alex' "
                                      "(the metric's default)")
        self.net = net
        self._weights = weights
        self._parts = {}
        _vgg.resolve_precision(precision)  # validates
        self.precision = precision  # the trunk's type: "auto" / "fp32" / "bf16" / "fp16" (see PerceptualLoss)

    def parts(self, device, dt: Optional[int] = None):
        if dt is None:
            dt = _vgg.resolve_precision(self.precision)
        key = (str(device), dt)
        if key not in self._parts and self.net == "alex":
            if self._weights is None:
                warnings.warn("LPIPS: pretrained AlexNet / lin weights are not available offline; using a deterministic "
                              "synthetic model", RuntimeWarning)
                feats = alex_synthetic_state_dict(0)
                g = torch.Generator().manual_seed(0)
                lins = {k: (torch.randn(c, generator=g) * 0.1).abs() for k, c in enumerate(ALEX_TAP_CH)}
            else:
                sd = torch.load(self._weights, map_location="cpu", weights_only=True) if isinstance(
                    self._weights, str) else dict(self._weights)
                feats, lins = _split_state_dict(sd)
            stack = AlexStack(device, feats, dtype=dt)
            self._parts[key] = (stack, [lins[k].to(device).float().contiguous() for k in range(5)])
        if key not in self._parts:
            if self._weights is None:
                warnings.warn("LPIPS: pretrained VGG16 / lin weights are not available offline; using a deterministic "
                              "synthetic model", RuntimeWarning)
                feats = _vgg.synthetic_state_dict(_vgg.VGG16_CFG, 30, seed=0)
                g = torch.Generator().manual_seed(0)
                lins = {k: (torch.randn(c, generator=g) * 0.1).abs() for k, c in enumerate(TAP_CH)}
            else:
                sd = torch.load(self._weights, map_location="cpu", weights_only=True) if isinstance(
                    self._weights, str) else dict(self._weights)
                feats, lins = _split_state_dict(sd)
            stack = _vgg.VGGStack(_vgg.VGG16_CFG, 30, device, feats, dtype=dt)
            self._parts[key] = (stack, [lins[k].to(device).float().contiguous() for k in range(5)])
        return self._parts[key]

    def value_and_grad(self, in0, in1, up: torch.Tensor, out: torch.Tensor, clamp: bool = True,
                       dt: Optional[int] = None) -> torch.Tensor:
        """Autograd-free form for the fused trainer: out[N] = LPIPS(clamp01(in0), clamp01(in1)) per image (the
        HybridLossPlus call on Bhat_srgb01 / B_srgb01), returns d(sum_n up[n] out[n]) / d in0 (through the clamp).
        Either backbone ('vgg': the reference's HybridLossPlus term, losses.py:268; 'alex': BASELINE.json cfg3's).
        `dt`: trunk dtype override (None: `precision`)."""
        stack, lins = self.parts(in0.device, dt)
        x0 = _vgg.prep_input(in0, SHIFT, SCALE, clamp=clamp, dtype=stack.dtype)
        x1 = _vgg.prep_input(in1, SHIFT, SCALE, clamp=clamp, dtype=stack.dtype)
        if isinstance(stack, AlexStack):
            t0, tape = stack.taps(x0, save=True)
            t1 = stack.taps(x1)
        else:
            _, tape, m0 = stack.forward(x0, save=True, taps=TAPS)
            _, _, m1 = stack.forward(x1, save=False, taps=TAPS)
            t0, t1 = [m0[t] for t in TAPS], [m1[t] for t in TAPS]
        grads = _tap_distances(stack, lins, t0, t1, out, True, up)
        return _vgg.input_grad(_trunk_backward(stack, tape, grads), in0, SCALE, clamp=clamp)

    def forward(self, in0, in1, retPerLayer: bool = False, normalize: bool = False):
        if retPerLayer:
            raise NotImplementedError("retPerLayer is not supported on MI355X")
        return _LPIPSFn.apply(in0, in1.to(in0.device), self, bool(normalize), _vgg.resolve_precision(self.precision))
