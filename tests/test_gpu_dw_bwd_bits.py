"""Bit pin of the fused depthwise backward (nbp_sca_sg_dw_bwd: SCA + SimpleGate backward + dw3x3 input / weight
gradients, the LDS-tiled dw_bwd_tiled kernel) across kernel rewrites: sha256 of dt1, dW and db on seeded inputs,
against tests/golden/dw_bwd_sha.json written by the kernel before the rewrite (`python tests/test_gpu_dw_bwd_bits.py
--write` on a GPU box).  Shapes: the cfg2 levels at small batches, ragged tiles (H % 16, W % 32 != 0), 16-column tiles
(W < 32) and the fp32 kernel; float64 parity of the same kernel is test_gpu_parity.py::test_dw_bwd_against_float64."""
import hashlib
import json
import os
import sys

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dw_bwd_sha.json")
SHAPES = [(2, 256, 256, 32), (3, 128, 128, 64), (2, 64, 64, 128), (4, 32, 32, 256), (3, 16, 16, 512), (2, 37, 45, 16),
          (1, 33, 70, 32), (5, 50, 96, 16), (3, 40, 33, 48), (2, 21, 19, 32)]
CASES = [(s, dt) for s in SHAPES for dt in (0, 1, 2)]


def _key(shape, dtype):
    return "x".join(map(str, shape)) + f"_dt{dtype}"


def _hashes(shape, dtype):
    import torch
    from lowlight_image_enhancement_amd._lib import call, query
    dev = torch.device("cuda:0")
    B, H, W, C = shape
    td = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[dtype]
    gen = torch.Generator(device=dev).manual_seed(B * 7 + H * W + C + dtype)
    M = B * H * W
    dh = torch.randn(M, C, device=dev, generator=gen).to(td)
    t1 = torch.randn(M, 2 * C, device=dev, generator=gen).to(td)
    t2 = torch.randn(M, 2 * C, device=dev, generator=gen).to(td)
    a = torch.randn(B, C, device=dev, generator=gen)
    ds = torch.randn(B, C, device=dev, generator=gen)
    w = torch.randn(2 * C, 9, device=dev, generator=gen)
    dt1 = torch.full((M, 2 * C), float("nan"), device=dev, dtype=td)
    dW, db = torch.empty(2 * C, 9, device=dev), torch.empty(2 * C, device=dev)
    ws = torch.empty(query("dw_bwd_workspace_floats", B, H, W, C), device=dev)
    call("sca_sg_dw_bwd", dh, a, ds, t2, t1, w, dt1, dW, db, ws, B, H, W, C, dtype)
    torch.cuda.synchronize()
    raw = [t.contiguous().view(torch.int16 if t.element_size() == 2 else torch.int32).cpu().numpy().tobytes() for t in (dt1, dW, db)]
    return [hashlib.sha256(r).hexdigest()[:32] for r in raw]


@pytest.mark.gpu
@pytest.mark.parametrize("shape,dtype", CASES, ids=[_key(s, d) for s, d in CASES])
def test_dw_bwd_bits_unchanged(dev, shape, dtype):
    gold = json.load(open(GOLD))
    assert _hashes(shape, dtype) == gold[_key(shape, dtype)]


if __name__ == "__main__" and "--write" in sys.argv:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    json.dump({_key(s, d): _hashes(s, d) for s, d in CASES}, open(GOLD, "w"), indent=1)
    print("wrote", GOLD)
