"""Per-rank sampling and loader construction for the SID input path.

Reference: NAFNet_base/basicsr/data/data_sampler.py (EnlargedSampler) and basicsr/data/__init__.py:63-141
(create_dataloader, worker_init_fn).  One process per GPU: each rank iterates its own shard of an epoch-seeded
permutation (no collective); the batches are converted on that rank's GPU by CUDAPrefetcher.
"""
from __future__ import annotations

import math
import random
from functools import partial

import numpy as np
import torch
from torch.utils.data.sampler import Sampler


class EnlargedSampler(Sampler):
    """EnlargedSampler(dataset, num_replicas, rank, ratio=1): rank's strided share of torch.randperm(total_size)
    (generator seeded with the epoch), indices taken modulo len(dataset)."""

    def __init__(self, dataset, num_replicas, rank, ratio=1):
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.num_samples = math.ceil(len(self.dataset) * ratio / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.epoch)
        indices = torch.randperm(self.total_size, generator=g).tolist()
        n = len(self.dataset)
        indices = [v % n for v in indices][self.rank:self.total_size:self.num_replicas]
        assert len(indices) == self.num_samples
        return iter(indices)

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch):
        self.epoch = epoch


def worker_init_fn(worker_id, num_workers, rank, seed):
    worker_seed = num_workers * rank + worker_id + seed
    np.random.seed(worker_seed)
    random.seed(worker_seed)


def create_dataloader(dataset, dataset_opt, num_gpu=1, dist=False, sampler=None, seed=None, rank=None):
    """basicsr create_dataloader: train -> batch_size_per_gpu (x num_gpu when not distributed), drop_last, shuffle
    unless a sampler is given, persistent workers when num_workers > 0; val / test -> batch 1.  prefetch_mode
    None / 'cuda' give a DataLoader whose batches CUDAPrefetcher converts on the GPU; 'cpu' (the reference's
    CPUPrefetcher of float tensors) is not offered, the float conversion being a device kernel here."""
    phase = dataset_opt["phase"]
    if rank is None:
        rank = torch.distributed.get_rank() if torch.distributed.is_available() and \
            torch.distributed.is_initialized() else 0
    if phase == "train":
        if dist:
            batch_size = dataset_opt["batch_size_per_gpu"]
            num_workers = dataset_opt["num_worker_per_gpu"]
        else:
            multiplier = 1 if num_gpu == 0 else num_gpu
            batch_size = dataset_opt["batch_size_per_gpu"] * multiplier
            num_workers = dataset_opt["num_worker_per_gpu"] * multiplier
        args = dict(dataset=dataset, batch_size=batch_size, shuffle=sampler is None, num_workers=num_workers,
                    sampler=sampler, drop_last=True, persistent_workers=num_workers > 0)
        args["worker_init_fn"] = partial(worker_init_fn, num_workers=num_workers, rank=rank, seed=seed) \
            if seed is not None else None
    elif phase in ("val", "test"):
        args = dict(dataset=dataset, batch_size=1, shuffle=False, num_workers=0)
    else:
        raise ValueError(f"Wrong dataset phase: {phase}. Supported ones are 'train', 'val' and 'test'.")
    args["pin_memory"] = dataset_opt.get("pin_memory", False)
    if dataset_opt.get("prefetch_mode") == "cpu":
        raise ValueError("prefetch_mode 'cpu' is not supported: SID batches are converted on the GPU "
                         "(use prefetch_mode 'cuda' with CUDAPrefetcher)")
    return torch.utils.data.DataLoader(**args)
