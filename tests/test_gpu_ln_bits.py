"""Bit pin of the NHWC LayerNorm2d kernels (nbp_ln_fwd_nhwc / nbp_ln_bwd_nhwc, arch_util.py:264-300) across load
restructuring: sha256 of the normalised output, the row stats, dx and the per-block weight / bias partial slabs on
seeded inputs, against tests/golden/ln_bits_sha.json written by the kernels before the change
(`python tests/test_gpu_ln_bits.py --write` on a GPU box).  Shapes: the cfg2 middle level (C 512), every lane-group
width, ragged row counts, channel counts that are not powers of two, the fp32 four-chunk lanes, with and without the
residual gradient; float64 parity of the same kernels is test_gpu_parity.py::test_ln_nhwc_any_channel_count."""
import hashlib
import json
import os
import sys

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ln_bits_sha.json")
SHAPES = [(4096, 512), (3001, 512), (1000, 40), (777, 96), (4097, 256), (513, 1024), (2049, 24), (65536, 32),
          (300, 2048), (1, 64)]
CASES = [(m, c, dt, r) for (m, c) in SHAPES for dt in (0, 1, 2) for r in (0, 1)
         if c % (4 if dt == 0 else 8) == 0 and c // (4 if dt == 0 else 8) <= 256]


def _key(case):
    m, c, dt, r = case
    return f"{m}x{c}_dt{dt}_res{r}"


def _hashes(case):
    import torch
    from lowlight_image_enhancement_amd._lib import call, query
    dev = torch.device("cuda:0")
    M, C, dt, res = case
    td = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[dt]
    gen = torch.Generator(device=dev).manual_seed(M * 3 + C + dt)
    x = (torch.randn(M, C, device=dev, generator=gen) * 2 + 0.3).to(td)
    w, b = torch.randn(C, device=dev, generator=gen), torch.randn(C, device=dev, generator=gen)
    n, st = torch.empty(M, C, device=dev, dtype=td), torch.empty(M, 2, device=dev)
    call("ln_fwd_nhwc", x, w, b, n, st, M, C, 1e-6, dt)
    dn = torch.randn(M, C, device=dev, generator=gen).to(td)
    dres = torch.randn(M, C, device=dev, generator=gen).to(td) if res else None
    dx = torch.empty(M, C, device=dev, dtype=td)
    slab = torch.full((2, query("ln_nhwc_grid", M, C, dt), C), float("nan"), device=dev)
    call("ln_bwd_nhwc", dn, x, st, w, dres, dx, slab[0], slab[1], M, C, dt)
    torch.cuda.synchronize()
    raw = [t.contiguous().view(torch.int16 if t.element_size() == 2 else torch.int32).cpu().numpy().tobytes()
           for t in (n, st, dx, slab)]
    return [hashlib.sha256(r).hexdigest()[:32] for r in raw]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[_key(c) for c in CASES])
def test_ln_bits_unchanged(dev, case):
    gold = json.load(open(GOLD))
    assert _hashes(case) == gold[_key(case)]


if __name__ == "__main__" and "--write" in sys.argv:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    json.dump({_key(c): _hashes(c) for c in CASES}, open(GOLD, "w"), indent=1)
    print("wrote", GOLD)
