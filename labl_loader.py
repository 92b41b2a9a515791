"""API-compatible module path of the reference LABL loader (Module_1/labl_loader(EXPERIMENTAL).py):
LABLShardedReader, PinnedRing, LABLPrefetcher - backed by the C++ mmap reader / hipHostMalloc ring /
producer thread (csrc/io/shard_io.cpp).  See crossscale_ecg/data/labl.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from crossscale_ecg.data.labl import LABLShardedReader, PinnedRing, LABLPrefetcher  # noqa: E402,F401

__all__ = ["LABLShardedReader", "PinnedRing", "LABLPrefetcher"]
