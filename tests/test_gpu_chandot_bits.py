"""Bit pin of the per-image channel dot (nbp_img_chan_dot: the SCA backward's da partials at levels 0/1,
NAFNet_arch.py:39-41) across load restructuring: sha256 of the chunk slab on seeded inputs, with and without the
second operand, against tests/golden/chandot_bits_sha.json written by the kernel before the change (`python
tests/test_gpu_chandot_bits.py --write` on a GPU box).  Shapes: cfg2 levels 0/1 at small batches, ragged chunks, C not
a multiple of 64, every dtype."""
import hashlib
import json
import os
import sys

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "chandot_bits_sha.json")
SHAPES = [(2, 256, 256, 32), (2, 128, 128, 64), (3, 37, 45, 16), (1, 64, 64, 96), (2, 33, 70, 128), (1, 16, 16, 512)]
CASES = [(s, dt, hy) for s in SHAPES for dt in (0, 1, 2) for hy in (1, 0)]


def _key(case):
    s, dt, hy = case
    return "x".join(map(str, s)) + f"_dt{dt}_y{hy}"


def _hashes(case):
    import torch
    from lowlight_image_enhancement_amd._lib import call, query
    dev = torch.device("cuda:0")
    (B, H, W, C), dt, hy = case
    td = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[dt]
    gen = torch.Generator(device=dev).manual_seed(B + H * W + C + dt)
    x = torch.randn(B * H * W, C, device=dev, generator=gen).to(td)
    y = torch.randn(B * H * W, C, device=dev, generator=gen).to(td) if hy else None
    chunks = query("dw_chunks", B, H, W, C, 0)
    slab = torch.full((B, chunks, C), float("nan"), device=dev)
    call("img_chan_dot", x, y, slab, B, H, W, C, dt)
    torch.cuda.synchronize()
    return [hashlib.sha256(slab.view(torch.int32).cpu().numpy().tobytes()).hexdigest()[:32]]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[_key(c) for c in CASES])
def test_chandot_bits_unchanged(dev, case):
    gold = json.load(open(GOLD))
    assert _hashes(case) == gold[_key(case)]


if __name__ == "__main__" and "--write" in sys.argv:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    json.dump({_key(c): _hashes(c) for c in CASES}, open(GOLD, "w"), indent=1)
    print("wrote", GOLD)
