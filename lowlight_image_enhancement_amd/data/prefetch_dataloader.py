"""CUDA prefetcher for the SID input path (reference: NAFNet_base/basicsr/data/prefetch_dataloader.py:90-132).

Same interface as the reference's CUDAPrefetcher (``CUDAPrefetcher(loader, opt)``, ``next()`` -> batch dict or None,
``reset()``): the next batch is uploaded on a side stream while the current step runs, and ``next()`` makes the
current stream wait for it.  The batches of SonySIDLMDBDataset carry the uint16 crop windows; on the side stream,
after the upload, ``nbp_sid_to_float`` (sid.hip) turns them into the reference's float32 NCHW tensors, so the step
receives the reference's batch dict.  Aliasing as in the reference: ``short`` and ``short_obs`` are ``lq``; ``long``
is ``gt``; ``long_raw`` has the values of ``gt`` (the same tensor here).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .._lib import call


def to_reference_batch(batch: Dict, device: torch.device) -> Dict:
    """Device batch dict from a collated uint16 batch, enqueued on the current stream (tensors moved with
    non_blocking=True: pinned host memory gives an asynchronous copy)."""
    out = {}
    for k, v in batch.items():
        if k in ("lq_u16", "gt_u16"):
            continue
        out[k] = v.to(device=device, non_blocking=True) if torch.is_tensor(v) else v
    s16 = batch["lq_u16"].to(device=device, non_blocking=True)
    l16 = batch["gt_u16"].to(device=device, non_blocking=True)
    if s16.shape != l16.shape or s16.dim() != 4 or s16.shape[3] != 3 or s16.dtype != torch.int16:
        raise ValueError(f"expected uint16 [B,H,W,3] crops, got {tuple(s16.shape)} / {tuple(l16.shape)}")
    B, H, W, _ = s16.shape
    ratio = out["expo_ratio"].reshape(B).to(torch.float32).contiguous()
    lq = torch.empty(B, 3, H, W, device=device)
    short_raw = torch.empty_like(lq)
    gt = torch.empty_like(lq)
    call("sid_to_float", s16, l16, ratio, B, H, W, lq, short_raw, gt)
    out.update({"lq": lq, "gt": gt, "short": lq, "long": gt, "short_raw": short_raw, "long_raw": gt,
                "short_obs": lq})
    return out


class CUDAPrefetcher:
    """CUDAPrefetcher(loader, opt): prefetches and converts the next batch on a side stream."""

    def __init__(self, loader, opt):
        self.ori_loader = loader
        self.loader = iter(loader)
        self.opt = opt
        if opt.get("num_gpu", 1) == 0 or not torch.cuda.is_available():
            raise RuntimeError("CUDAPrefetcher: the SID input path converts batches on the GPU (num_gpu > 0)")
        self.stream = torch.cuda.Stream()
        self.device = torch.device("cuda")
        self.preload()

    def preload(self) -> None:
        try:
            raw = next(self.loader)
        except StopIteration:
            self.batch = None
            return
        with torch.cuda.stream(self.stream):
            self.batch = to_reference_batch(raw, self.device)

    def next(self) -> Optional[Dict]:
        cur = torch.cuda.current_stream()
        cur.wait_stream(self.stream)
        batch = self.batch
        if batch is not None:
            for v in batch.values():  # allocated on the side stream, consumed on the current one
                if torch.is_tensor(v) and v.is_cuda:
                    v.record_stream(cur)
        self.preload()
        return batch

    def reset(self) -> None:
        self.loader = iter(self.ori_loader)
        self.preload()
