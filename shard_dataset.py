"""API-compatible module path of the reference ``shard_dataset`` (Module_3/shard_dataset.py):
assign_shards_evenly, load_shard, ShardDataset, make_dataloader, load_shards_to_gpu, make_gpu_batch_iter."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from crossscale_ecg.data.shards import assign_shards_evenly, load_shard  # noqa: E402,F401
from crossscale_ecg.data.dataset import (ShardDataset, make_dataloader, load_shards_to_gpu,  # noqa: E402,F401
                                         make_gpu_batch_iter, DeviceIndexSampler)

__all__ = ["assign_shards_evenly", "load_shard", "ShardDataset", "make_dataloader", "load_shards_to_gpu",
           "make_gpu_batch_iter", "DeviceIndexSampler"]
