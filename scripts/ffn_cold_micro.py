"""Cold-weight probe of the row-stationary FFN launches at the middle level (C 512, 16^2, bs 16, fp16): a graph of 12
launches over the SAME weights / activations (the micro's L2-warm case) against 12 launches over 12 distinct weight sets
(and distinct activations), as in the step's chain of blocks.  Per launch, µs.
    python scripts/ffn_cold_micro.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_ffn_rows import _fused, _operands, _reference  # noqa: E402
from c1dw_tile_micro import graph_time  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    dt, C, hw, B, NB = 2, 512, 256, 16, 12
    M = B * hw
    sets = [_operands(dev, dt, B, hw, C, 1 + i) for i in range(NB)]
    ref = _reference(dev, dt, M, C, hw, sets[0], True)
    outs = [{k: (torch.empty_like(v) if v is not None else None) for k, v in ref.items()} for _ in range(NB)]
    # distinct weights, shared activations
    wsets = [dict(sets[0], **{k: s[k] for k in ("w3", "w4", "w5")}) for s in sets]
    for s in wsets:
        s.pop("f3", None)

    def same():
        for i in range(NB):
            _fused(dev, dt, M, C, hw, sets[0], True, outs[0])

    def dist_w():
        for i in range(NB):
            _fused(dev, dt, M, C, hw, wsets[i], True, outs[0])

    def dist_all():
        for i in range(NB):
            _fused(dev, dt, M, C, hw, sets[i], True, outs[i])
    # distinct activations in, shared outputs / shared inputs, distinct outputs
    isets = [dict(s, **{k: sets[0][k] for k in ("w3", "w4", "w5")}) for s in sets]
    for s in isets:
        s.pop("f3", None)

    def dist_in():
        for i in range(NB):
            _fused(dev, dt, M, C, hw, isets[i], True, outs[0])

    def dist_out():
        for i in range(NB):
            _fused(dev, dt, M, C, hw, sets[0], True, outs[i])
    for name, fn in (("same", same), ("distinct weights", dist_w), ("distinct inputs", dist_in),
                     ("distinct outputs", dist_out), ("distinct all", dist_all)):
        t = min(graph_time(fn, iters) for _ in range(3)) / NB
        print(f"ffn_rows_fwd<512> x{NB}, {name}: {t:.1f} us per launch", flush=True)


if __name__ == "__main__":
    main()
