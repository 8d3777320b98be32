"""Per-workgroup timeline of the deep-level 1x1-conv GEMMs, from the probe library
(scripts/build_probe.py: gemm_glds_kernel stamps s_memrealtime, 100 MHz, at entry / prologue DMAs issued / K-tile 0
landed / last MFMA issued / epilogue stores landed, plus HW_ID / XCC_ID).  Per shape: event time per launch
(back-to-back), then one warm launch's stamps: phase percentiles over workgroups (us) and the kernel span.
    NBP_LIB=$PWD/lowlight_image_enhancement_amd/_lib/probe/liblowlight_nbp.so python scripts/gemm_timeline.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd._lib import call, lib  # noqa: E402

WORDS = 16384 * 8


def read(dll):
    buf = (ctypes.c_ulonglong * WORDS)()
    n = dll.nbp_gemm_probe_read(buf, WORDS)
    assert n == WORDS, n
    return np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).copy()


def pct(x):
    return "p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))


def main():
    dll = lib().dll
    assert hasattr(dll, "nbp_gemm_probe_read"), "not the probe library (NBP_LIB)"
    dev = torch.device("cuda:0")
    TD = torch.float16
    out = []
    for M, C in ((4096, 512), (16384, 256)):
        for N, K in ((2 * C, C), (C, C), (C, 2 * C)):
            A = torch.randn(M, K, device=dev).to(TD)
            W = (torch.randn(N, K, device=dev) / K ** 0.5).to(TD)
            Cm = torch.empty(M, N, device=dev, dtype=TD)

            def run():
                call("gemm_bf16", A, K, 0, None, 256, 2, W, K, Cm, N, 0, 2, M, N, K, 0, 0, 0, None, None, None, None)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                run()
            e1.record()
            torch.cuda.synchronize()
            ev = e0.elapsed_time(e1) * 1e3 / 50
            before = read(dll)
            run()
            torch.cuda.synchronize()
            after = read(dll)
            rows = np.nonzero((after[:, 0] != before[:, 0]))[0]
            s = after[rows].astype(np.int64)
            t = (s[:, :6] - s[:, 0].min()) * 0.01  # us
            hw, xcc = s[:, 6], s[:, 7] & 0xF
            cu = (xcc << 8) | ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5)
            ucu, inv = np.unique(cu, return_inverse=True)
            per_cu = np.bincount(inv)
            # start of the first / second workgroup on each CU
            first = np.full(len(ucu), np.inf)
            second = np.full(len(ucu), np.inf)
            for k in np.argsort(t[:, 0]):
                c = inv[k]
                if first[c] == np.inf:
                    first[c] = t[k, 0]
                elif second[c] == np.inf:
                    second[c] = t[k, 0]
            out.append(f"M={M} N={N} K={K}: {ev:.2f} us/launch (events, back-to-back); {len(rows)} workgroups on "
                       f"{len(ucu)} CUs ({per_cu.min()}-{per_cu.max()} per CU), kernel span {t[:, 5].max():.2f} us")
            out.append(f"  start          {pct(t[:, 0])}")
            out.append(f"  1st WG per CU  {pct(first)}")
            if np.isfinite(second).any():
                out.append(f"  2nd WG per CU  {pct(second[np.isfinite(second)])}")
            out.append(f"  args in regs   {pct(t[:, 1] - t[:, 0])}")
            out.append(f"  prologue issue {pct(t[:, 2] - t[:, 1])}")
            out.append(f"  K-tile 0 land  {pct(t[:, 3] - t[:, 2])}")
            out.append(f"  rest of K loop {pct(t[:, 4] - t[:, 3])}")
            out.append(f"  epilogue       {pct(t[:, 5] - t[:, 4])}")
            out.append(f"  workgroup life {pct(t[:, 5] - t[:, 0])}")
            xs = []
            for x in range(8):
                sel = xcc == x
                if sel.any():
                    xs.append(f"{x}:{t[sel, 0].min():.2f}/{np.median(t[sel, 0]):.2f}/{t[sel, 0].max():.2f}")
            out.append("  start by XCC (min/med/max) " + "  ".join(xs))
            n_out = 12 if np.isfinite(second).any() else 11
            print("\n".join(out[-n_out:]), flush=True)


if __name__ == "__main__":
    main()
