"""pebble_amd — MI355X-native decoder for Pebble SSTable data blocks.

The hot path (raw data blocks in HBM -> flat key / value / offset arrays) runs in
hand-written gfx950 HIP kernels inside libpebble_amd.so, reached through the
C-ABI declared in include/pebble_amd.h.  This package is the host layer:

  pebble_amd.batch   BlockBatch / decode() / DecodedBatch (device buffers, streams)
  pebble_amd.rowblk  Writer, NewIter/Iter mirroring sstable/rowblk
  pebble_amd.shard   multi-GPU sharding + RCCL offset concat
"""
from . import _native  # noqa: F401

__all__ = ["batch", "rowblk", "build"]
