"""SID input path: LMDB / disk PNG16 -> uint16 crops (native host code) -> the reference's
float32 batch on the GPU (HIP), behind the reference's dataset / prefetcher interface."""
from .data_sampler import EnlargedSampler, create_dataloader, worker_init_fn
from .file_client import FileClient, LmdbBackend, expand_with_sid_root
from .prefetch_dataloader import CUDAPrefetcher, to_reference_batch
from .sony_sid_lmdb_dataset import MAX_16BIT_VALUE, SonySIDLMDBDataset, decode_batch, png_shape

__all__ = ["EnlargedSampler", "create_dataloader", "worker_init_fn", "FileClient", "LmdbBackend", "expand_with_sid_root", "CUDAPrefetcher", "to_reference_batch",
           "MAX_16BIT_VALUE", "SonySIDLMDBDataset", "decode_batch", "png_shape"]
