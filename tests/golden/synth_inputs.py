"""Synthetic input batches shared by the golden generator (make_golden.py) and the GPU tests.

Test infrastructure only: the generator runs the reference on these batches in the build container; the tests
regenerate the same batches from the seed on the GPU box (numpy PCG64: bit-identical on every platform).
"""
from __future__ import annotations

import numpy as np


def cfg5_inputs(seed=500, N=8, H=1024, W=1024):
    """Synthetic RAW batch of BASELINE configs[4]: 12-bit sensor values q / 4095, exposure ratios from
    {100, 250, 300}; pred = the long exposure scaled down by the ratio, obs = an independent 12-bit draw around it.
    numpy PCG64 integers: bit-identical on every platform (the test regenerates them from the seed)."""
    rng = np.random.default_rng(seed)
    ratios = rng.choice(np.asarray([100.0, 250.0, 300.0], dtype=np.float32), size=N)
    ql = rng.integers(0, 4096, size=(N, 3, H, W), dtype=np.uint16)
    noise = rng.integers(-64, 65, size=(N, 3, H, W), dtype=np.int16)
    qs = np.clip(ql.astype(np.int32) + noise, 0, 4095).astype(np.uint16)
    pred = (ql.astype(np.float32) / np.float32(4095.0)) / ratios[:, None, None, None]
    obs = qs.astype(np.float32) / np.float32(4095.0)
    return pred.astype(np.float32), obs, ratios, int(ql.astype(np.int64).sum()), int(qs.astype(np.int64).sum())
