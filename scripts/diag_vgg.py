"""Diagnostic: VGG input-gradient error vs depth, against float64 torch and against a torch emulation that rounds
stored activations / gradients to bf16 at the same points as the kernels (distinguishes precision from bugs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as Fn

from lowlight_image_enhancement_amd._lib import call
from lowlight_image_enhancement_amd.vgg import VGG19_CFG, VGGStack, _layers, input_grad, prep_input, synthetic_state_dict

dev = torch.device("cuda")
bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731


def torch_stack(sd, x, n, round_bf16):
    h = x
    for kind, idx, _, _ in _layers(VGG19_CFG, n):
        if kind == "pool":
            h = Fn.max_pool2d(h, 2)
        else:
            h = Fn.relu(Fn.conv2d(h, sd[f"{idx}.weight"].double(), sd[f"{idx}.bias"].double(), padding=1))
            if round_bf16:
                h = RoundBF16.apply(h)
    return h


class RoundBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return bf(x)

    @staticmethod
    def backward(ctx, g):
        return bf(g)


def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm()).item()


sd = synthetic_state_dict(VGG19_CFG, 36, 0)
sd = {k: (v + 0.01 if k.endswith("bias") else v) for k, v in sd.items()}
sdb = {k: (bf(v) if k.endswith("weight") else v.double()) for k, v in sd.items()}
g = torch.Generator().manual_seed(2)
gen = torch.rand(2, 3, 64, 48, generator=g)
tgt = torch.rand(2, 3, 64, 48, generator=g)
mean = torch.tensor([0.485, 0.456, 0.406], dtype=torch.float64).view(1, 3, 1, 1)
std = torch.tensor([0.229, 0.224, 0.225], dtype=torch.float64).view(1, 3, 1, 1)
for dt, scale in ((1, 1.0), (2, 65536.0)):  # fp16 under the trainer's initial loss scale (GradScaler's 2^16)
    for n in (4, 9, 18, 27, 36):
        st = VGGStack(VGG19_CFG, n, dev, sd, dtype=dt)
        x = gen.to(dev)
        fg, tape, _ = st.forward(prep_input(x, dtype=dt), save=True)
        ft, _, _ = st.forward(prep_input(tgt.to(dev), dtype=dt), save=False)
        d = torch.empty_like(fg)
        up = torch.full((1,), scale, device=dev)
        call("feat_dist_bwd", fg, ft, fg.numel(), 0, 1.0 / fg.numel(), 1, up, d, dt)
        dx = input_grad(st.backward(tape, d), x) / scale
        res = []
        for rb in ((False, True) if dt == 1 else (False,)):
            xr = gen.double().requires_grad_(True)
            xin = (xr.clamp(0, 1) - mean) / std
            if rb:
                xin = RoundBF16.apply(xin)
            fr = torch_stack(sdb if rb else sd, xin, n, rb)
            with torch.no_grad():
                xt = (tgt.double() - mean) / std
                ftr = torch_stack(sdb if rb else sd, bf(xt) if rb else xt, n, rb)
            Fn.mse_loss(fr, ftr).backward()
            res.append(rel(dx, xr.grad))
        fe = rel(fg.float(), torch_stack(sd, (gen.double() - mean) / std, n, False).permute(0, 2, 3, 1))
        emu = f"  vs bf16-emulation {res[1]:.4f}" if len(res) > 1 else ""
        print(f"{'bf16' if dt == 1 else 'fp16'} features[:{n}]: feat rel err vs fp64 {fe:.4f}  grad rel err vs fp64 "
              f"{res[0]:.4f}{emu}", flush=True)
