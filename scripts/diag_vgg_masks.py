"""Count ReLU-mask and max-pool-argmax disagreements between the fp32 GPU VGG16 forward and float64 torch."""
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd.vgg import VGG16_CFG, VGGStack, _layers, prep_input, synthetic_state_dict  # noqa: E402

dev = torch.device("cuda:0")
feats = synthetic_state_dict(VGG16_CFG, 30, seed=1)
g = torch.Generator().manual_seed(3)
x0 = torch.rand(2, 3, 64, 64, generator=g)
st = VGGStack(VGG16_CFG, 30, dev, feats, dtype=0)
x8 = prep_input(x0.to(dev), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0), clamp=False, dtype=0)
last, tape, _ = st.forward(x8, save=True)
h = x0.double()
ti = 0
for kind, idx, _, _ in _layers(VGG16_CFG, 30):
    rec = tape[ti]
    ti += 1
    if kind == "pool":
        hp, ind = Fn.max_pool2d(h, 2, return_indices=True)
        gidx = rec[2].cpu().long().permute(0, 3, 1, 2)  # window position 0..3
        H, W = h.shape[2], h.shape[3]
        oi = torch.arange(hp.shape[2]).view(1, 1, -1, 1)
        oj = torch.arange(hp.shape[3]).view(1, 1, 1, -1)
        flat = ind  # index into H*W
        pos = ((flat // W) - 2 * oi) * 2 + ((flat % W) - 2 * oj)
        nonzero = hp > 0
        mism = ((pos != gidx) & nonzero).sum().item()
        print(f"pool {idx}: argmax mismatches (max > 0) {mism} of {int(nonzero.sum())}")
        h = hp
    else:
        pre = Fn.conv2d(h, feats[f"{idx}.weight"].double(), feats[f"{idx}.bias"].double(), padding=1)
        y = rec[3].double().cpu().permute(0, 3, 1, 2)
        flips = ((pre > 0) != (y > 0)).sum().item()
        near = (pre.abs() < 1e-5 * pre.abs().max()).sum().item()
        print(f"conv {idx}: relu mask flips {flips} of {pre.numel()} (|pre| < 1e-5 max: {near}); max rel err "
              f"{((y - pre.clamp_min(0)).abs().max() / pre.abs().max()).item():.2e}")
        h = pre.clamp_min(0)
