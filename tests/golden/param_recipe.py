"""Deterministic parameter recipe shared by the golden generator and the parity tests.

Test infrastructure only.  The reference initialises NAFBlock beta/gamma to zero
(NAFNet_arch.py:56-57), which makes every block an identity; parity runs instead
fill every tensor of a state_dict from one seeded generator, walking the keys in
state_dict order, so both the reference model (in make_golden.py) and the MI355X
model (in tests/) can be given bit-identical weights from a seed alone.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Tuple

import torch


def recipe_tensor(name: str, shape: Tuple[int, ...], gen: torch.Generator) -> torch.Tensor:
    shape = tuple(int(s) for s in shape)
    z = torch.randn(shape, generator=gen, dtype=torch.float32)
    leaf = name.rsplit(".", 1)[-1]
    if leaf in ("beta", "gamma"):
        return z * 0.2
    if ".norm" in name and leaf == "weight":
        return 1.0 + 0.1 * z
    if leaf == "bias":
        return 0.05 * z
    if leaf == "weight" and len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        return z * (1.0 / math.sqrt(fan_in))
    return 0.1 * z


def recipe_state(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int) -> Dict[str, torch.Tensor]:
    gen = torch.Generator().manual_seed(seed)
    return {n: recipe_tensor(n, s, gen) for n, s in named_shapes}
