"""Per-shape timing of the bf16 GEMM / wgrad launches at the NAFNet deep levels (microbenchmark, HIP events over
repeated launches on resident operands).  python scripts/gemm_micro.py  (env knobs such as NBP_GEMM_MINBLK apply)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, query  # noqa: E402

dev = torch.device("cuda:0")
REPS = 200
DT = int(os.environ.get("NBP_MICRO_DT", "1"))  # 1 bf16, 2 fp16
TD = torch.float16 if DT == 2 else torch.bfloat16


def timeit(fn):
    """GPU time per launch: REPS launches captured in one HIP graph and replayed (no host dispatch in the clock)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(REPS):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS * 1e3


rows = []
for (M, N, K, mode) in [(4096, 1024, 512, 0), (4096, 512, 512, 0), (4096, 512, 512, 2), (4096, 512, 1024, 0),
                        (16384, 512, 256, 0), (16384, 256, 256, 0), (16384, 256, 512, 0), (65536, 256, 128, 0),
                        (65536, 128, 128, 0), (65536, 128, 256, 0)]:
    A = torch.randn(M, K, device=dev).to(TD)
    W = torch.randn(N, K, device=dev).to(TD)
    Cc = torch.empty(M, N, device=dev, dtype=TD)
    bias = torch.randn(N, device=dev)
    sc = torch.rand(M // 256 + 1, K, device=dev)
    us = timeit(lambda: call("gemm_bf16", A, K, mode, sc if mode == 2 else None, 256, DT, W, K, Cc, N, 0, DT, M, N, K,
                             0, 0, 0, bias, None, None, None))
    fl = 2.0 * M * N * K
    rows.append(f"gemm  M={M:6d} N={N:5d} K={K:5d} amode={mode}: {us:7.2f} us  {fl / us / 1e6:7.1f} TF")
for (M, N, K) in [(4096, 1024, 512), (4096, 512, 512), (16384, 512, 256), (16384, 256, 256), (65536, 256, 128)]:
    G = torch.randn(M, N, device=dev).to(TD)
    X = torch.randn(M, K, device=dev).to(TD)
    dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    n_ws = query("wgrad_workspace_floats", M, N, K)
    ws = torch.empty(n_ws, device=dev)
    us = timeit(lambda: call("wgrad_f32", G, N, 0, X, K, 0, None, 1, M, N, K, 0, 0, 0, 0, dW, db, ws, n_ws, DT))
    rows.append(f"wgrad M={M:6d} N={N:5d} K={K:5d} (+reduce): {us:7.2f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF")
print(f"NBP_GEMM_MINBLK={os.environ.get('NBP_GEMM_MINBLK', '-')}")
print("\n".join(rows))

# reference point: the vendor library (torch.mm -> hipBLASLt / rocBLAS) on the same shapes, bf16 in / out
ref = []
for (M, N, K) in [(4096, 1024, 512), (4096, 512, 512), (16384, 512, 256), (16384, 256, 256), (65536, 256, 128),
                  (65536, 128, 128)]:
    A = torch.randn(M, K, device=dev).to(TD)
    W = torch.randn(N, K, device=dev).to(TD)
    us = timeit(lambda: torch.mm(A, W.t()))
    ref.append(f"torch.mm M={M:6d} N={N:5d} K={K:5d}: {us:7.2f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF")
    # an empty-ish launch for the launch floor
z = torch.empty(256, device=dev)
ref.append(f"launch floor (tiny fill): {timeit(lambda: z.fill_(1.0)):.2f} us")
print("\n".join(ref))
