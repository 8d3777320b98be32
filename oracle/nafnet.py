"""Oracle: NAFNet (Scenario B) forward, functional over a reference-named state dict.

Test infrastructure only (see oracle/__init__.py).  Backward comes from autograd
over these ops, except LayerNorm2d whose hand-written backward is restated too.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F


class _LN2d(torch.autograd.Function):
    """LayerNormFunction (NAFNet_base/basicsr/models/archs/arch_util.py:264-289)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        mu = x.mean(1, keepdim=True)
        var = (x - mu).pow(2).mean(1, keepdim=True)
        y = (x - mu) / (var + eps).sqrt()
        ctx.save_for_backward(y, var, w)
        ctx.eps = eps
        C = x.shape[1]
        return w.view(1, C, 1, 1) * y + b.view(1, C, 1, 1)

    @staticmethod
    def backward(ctx, dy):
        y, var, w = ctx.saved_tensors
        C = dy.shape[1]
        g = dy * w.view(1, C, 1, 1)
        mg = g.mean(dim=1, keepdim=True)
        mgy = (g * y).mean(dim=1, keepdim=True)
        dx = 1.0 / torch.sqrt(var + ctx.eps) * (g - y * mgy - mg)
        return dx, (dy * y).sum(dim=(0, 2, 3)), dy.sum(dim=(0, 2, 3)), None


def layer_norm2d(x, w, b, eps=1e-6):
    return _LN2d.apply(x, w, b, eps)


def nafblock(P: Dict[str, torch.Tensor], pre: str, inp: torch.Tensor) -> torch.Tensor:
    """NAFBlock.forward (NAFNet_arch.py:59-80); dropout is Identity at rate 0 (:53-54)."""
    c = inp.shape[1]
    x = layer_norm2d(inp, P[pre + "norm1.weight"], P[pre + "norm1.bias"])
    x = F.conv2d(x, P[pre + "conv1.weight"], P[pre + "conv1.bias"])
    x = F.conv2d(x, P[pre + "conv2.weight"], P[pre + "conv2.bias"], padding=1, groups=2 * c)
    x = x[:, :c] * x[:, c:]  # SimpleGate (:22-25)
    s = F.adaptive_avg_pool2d(x, 1)  # SCA (:37-41)
    s = F.conv2d(s, P[pre + "sca.1.weight"], P[pre + "sca.1.bias"])
    x = x * s
    x = F.conv2d(x, P[pre + "conv3.weight"], P[pre + "conv3.bias"])
    y = inp + x * P[pre + "beta"]
    x = layer_norm2d(y, P[pre + "norm2.weight"], P[pre + "norm2.bias"])
    x = F.conv2d(x, P[pre + "conv4.weight"], P[pre + "conv4.bias"])
    x = x[:, :c] * x[:, c:]
    x = F.conv2d(x, P[pre + "conv5.weight"], P[pre + "conv5.bias"])
    return y + x * P[pre + "gamma"]


def nafnet(P: Dict[str, torch.Tensor], inp: torch.Tensor, enc_blk_nums: Sequence[int], middle_blk_num: int,
           dec_blk_nums: Sequence[int]) -> torch.Tensor:
    """NAFNet.forward (NAFNet_arch.py:132-162)."""
    B, C, H, W = inp.shape
    pad = 2 ** len(enc_blk_nums)
    ph, pw = (pad - H % pad) % pad, (pad - W % pad) % pad
    inp = F.pad(inp, (0, pw, 0, ph))
    x = F.conv2d(inp, P["intro.weight"], P["intro.bias"], padding=1)
    encs: List[torch.Tensor] = []
    for i, n in enumerate(enc_blk_nums):
        for j in range(n):
            x = nafblock(P, f"encoders.{i}.{j}.", x)
        encs.append(x)
        x = F.conv2d(x, P[f"downs.{i}.weight"], P[f"downs.{i}.bias"], stride=2)
    for j in range(middle_blk_num):
        x = nafblock(P, f"middle_blks.{j}.", x)
    for i, n in enumerate(dec_blk_nums):
        x = F.pixel_shuffle(F.conv2d(x, P[f"ups.{i}.0.weight"]), 2)
        x = x + encs[::-1][i]
        for j in range(n):
            x = nafblock(P, f"decoders.{i}.{j}.", x)
    x = F.conv2d(x, P["ending.weight"], P["ending.bias"], padding=1)
    x = x + inp
    return x[:, :, :H, :W]


def nafnet_param_shapes(img_channel=3, width=16, middle_blk_num=1, enc_blk_nums=(), dec_blk_nums=()):
    """Reference state_dict keys and shapes in registration order (NAFNet_arch.py:85-130)."""
    out = [("intro.weight", (width, img_channel, 3, 3)), ("intro.bias", (width,)),
           ("ending.weight", (img_channel, width, 3, 3)), ("ending.bias", (img_channel,))]

    def block(pre, c):
        return [(pre + "beta", (1, c, 1, 1)), (pre + "gamma", (1, c, 1, 1)),
                (pre + "conv1.weight", (2 * c, c, 1, 1)), (pre + "conv1.bias", (2 * c,)),
                (pre + "conv2.weight", (2 * c, 1, 3, 3)), (pre + "conv2.bias", (2 * c,)),
                (pre + "conv3.weight", (c, c, 1, 1)), (pre + "conv3.bias", (c,)),
                (pre + "sca.1.weight", (c, c, 1, 1)), (pre + "sca.1.bias", (c,)),
                (pre + "conv4.weight", (2 * c, c, 1, 1)), (pre + "conv4.bias", (2 * c,)),
                (pre + "conv5.weight", (c, c, 1, 1)), (pre + "conv5.bias", (c,)),
                (pre + "norm1.weight", (c,)), (pre + "norm1.bias", (c,)),
                (pre + "norm2.weight", (c,)), (pre + "norm2.bias", (c,))]

    chan = width
    enc = []
    downs = []
    for i, n in enumerate(enc_blk_nums):
        for j in range(n):
            enc += block(f"encoders.{i}.{j}.", chan)
        downs += [(f"downs.{i}.weight", (2 * chan, chan, 2, 2)), (f"downs.{i}.bias", (2 * chan,))]
        chan *= 2
    mid = []
    for j in range(middle_blk_num):
        mid += block(f"middle_blks.{j}.", chan)
    dec = []
    ups = []
    for i, n in enumerate(dec_blk_nums):
        ups += [(f"ups.{i}.0.weight", (2 * chan, chan, 1, 1))]
        chan //= 2
        for j in range(n):
            dec += block(f"decoders.{i}.{j}.", chan)
    # nn.Module registration order: intro, ending, encoders, decoders, middle_blks, ups, downs
    return out + enc + dec + mid + ups + downs
