"""SID input path throughput: native PNG16 decode + crop on host threads, the pinned uint16
upload and the device conversion (nbp_sid_to_float), at SID sRGB size (2848 x 4256 x 3, 16-bit) with 512 x 512
training crops, batch 16.  Synthetic images (smooth gradients + noise, Up-filtered, zlib level 6)."""
import argparse
import os
import sys
import time
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def png16(img: np.ndarray) -> bytes:
    import struct
    H, W, _ = img.shape
    be = img.astype(">u2").view(np.uint8).reshape(H, W * 6)
    up = be.astype(np.int16)
    up[1:] -= be[:-1].astype(np.int16)
    rows = np.concatenate([np.full((H, 1), 2, np.uint8), (up & 255).astype(np.uint8)], 1)
    rows[0, 0] = 0
    rows[0, 1:] = be[0]

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d))
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 16, 2, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(rows.tobytes(), 6)) + chunk(b"IEND", b""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--H", type=int, default=2848)
    ap.add_argument("--W", type=int, default=4256)
    ap.add_argument("--ps", type=int, default=512)
    args = ap.parse_args()
    from lowlight_image_enhancement_amd._lib import call
    from lowlight_image_enhancement_amd.data.sony_sid_lmdb_dataset import decode_batch
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:args.H, 0:args.W]
    pngs = []
    for i in range(4):
        img = np.stack([(yy * 7 + xx * 3 + 997 * c + 1000 * i) % 60000 for c in range(3)], -1)
        img = (img + rng.integers(0, 256, img.shape)).astype(np.uint16)
        pngs.append(png16(img))
    bufs = [pngs[i % 4] for i in range(2 * args.images)]
    wins = [(int(rng.integers(0, args.H - args.ps + 1)), int(rng.integers(0, args.W - args.ps + 1)), args.ps, args.ps)
            for _ in range(args.images)] * 2
    decode_batch(bufs[:2], wins[:2], 2)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        u16 = decode_batch(bufs, wins, args.threads)
    t_dec = (time.perf_counter() - t0) / reps
    B, ps = args.images, args.ps
    res = {"png_bytes_mean": int(np.mean([len(p) for p in pngs])), "decode_threads": args.threads,
           "decode_ms_per_batch": round(t_dec * 1e3, 2), "decode_pairs_per_s": round(B / t_dec, 1)}
    if torch.cuda.is_available():
        dev = torch.device("cuda")
        host = torch.from_numpy(u16.view(np.int16)).pin_memory()
        d16 = torch.empty_like(host, device=dev)
        ratio = torch.full((B,), 100.0, device=dev)
        lq, sr, lr = (torch.empty(B, 3, ps, ps, device=dev) for _ in range(3))
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for _ in range(3):
            d16.copy_(host, non_blocking=True)
            call("sid_to_float", d16[:B], d16[B:], ratio, B, ps, ps, lq, sr, lr)
        torch.cuda.synchronize()
        e[0].record()
        for _ in range(10):
            d16.copy_(host, non_blocking=True)
        e[1].record()
        for _ in range(10):
            call("sid_to_float", d16[:B], d16[B:], ratio, B, ps, ps, lq, sr, lr)
        e[2].record()
        torch.cuda.synchronize()
        h2d = e[0].elapsed_time(e[1]) / 10
        k = e[1].elapsed_time(e[2]) / 10
        kbytes = B * ps * ps * 3 * (2 * 2 + 3 * 4)
        res.update({"h2d_ms_per_batch": round(h2d, 3), "h2d_GBps": round(host.numel() * 2 / h2d / 1e6, 1),
                    "convert_us_per_batch": round(k * 1e3, 1), "convert_GBps": round(kbytes / k / 1e6, 1),
                    "convert_hbm_frac": round(kbytes / k / 1e6 / 8000, 3)})
    print(res, flush=True)


if __name__ == "__main__":
    main()
