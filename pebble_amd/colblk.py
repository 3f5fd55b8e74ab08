"""Host-side mirror of Pebble's sstable/colblk data-block API over the device decoder.

  DataBlockEncoder — colblk.DataBlockEncoder (sstable/colblk/data_block.go:600-790)
                     with colblk.DefaultKeySchema or cockroachkvs.KeySchema ("crdb1"),
                     native (libpebble_amd.so), byte-exact with the reference
  NewDataBlockIter — DataBlockDecoder.Init + DataBlockIter.Init (data_block.go:1096-1109,
                     1288-1368): the block is decoded on the GPU, the iterator then
                     walks the flat decoded arrays (rowblk.Iter semantics: First/Next/
                     Last/Prev/SeekGE/SeekLT, SyntheticSeqNum, HideObsoletePoints)
  gen_col_blocks   — seeded synthetic config-3 batches (cockroachkvs.KeyGenConfig)

A block whose metadata init would panic in Go raises CorruptionError, as
InitDataBlockMetadata converts that panic (data_block.go:1001-1014).
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np

from . import _native as N
from .rowblk import CorruptionError, Iter, Transforms, bytes_compare, kvs_of_block

SCHEMA_DEFAULT = N.PBL_FMT_COL_DEFAULT
SCHEMA_CRDB1 = N.PBL_FMT_COL_CRDB1

VALUE_IN_PLACE, VALUE_BLOCK_HANDLE, VALUE_BLOB_HANDLE = 0, 1, 2


class DataBlockEncoder:
    """colblk.DataBlockEncoder.  `add` performs KeyWriter.ComparePrev itself and
    returns KeyComparison.PrefixEqual()."""

    def __init__(self, schema: int = SCHEMA_CRDB1, bundle_size: int = 16, tiering: bool = False):
        """`tiering`: Init(schema, WithTieringColumns()) -- the Pebblev8 layout
        (sstable/format.go:305-316), whose add() also takes a base.KVMeta."""
        self._lib = N.gen_lib()
        self._w = self._lib.pbl_colblk_writer_new(schema, bundle_size)
        if not self._w:
            raise ValueError(f"bad schema {schema} / bundle size {bundle_size}")
        self.schema = schema
        self.tiering = tiering
        if tiering:
            self._lib.pbl_colblk_writer_set_tiering(self._w, 1)

    def __del__(self):
        w, self._w = getattr(self, "_w", None), None
        if w:
            self._lib.pbl_colblk_writer_free(w)

    def reset(self) -> None:
        self._lib.pbl_colblk_writer_reset(self._w)

    def add(self, user_key: bytes, trailer: int, value: bytes = b"", value_kind: int = VALUE_IN_PLACE,
            is_obsolete: bool = False, prefix_len: int = -1, meta: tuple = (0, 0),
            secondary_handle: bytes = b"") -> bool:
        """Add / AddWithSecondaryBlobHandle (data_block.go:694-765); `meta` is
        (TieringSpanID, TieringAttribute), stored when the attribute is set."""
        r = self._lib.pbl_colblk_writer_add_meta(self._w, user_key, len(user_key), prefix_len, trailer, value,
                                                len(value), value_kind, int(is_obsolete), int(meta[0]),
                                                int(meta[1]), secondary_handle, len(secondary_handle))
        if r not in (0, 1):
            raise ValueError(f"invalid key {user_key!r}")
        return bool(r)

    def rows(self) -> int:
        return int(self._lib.pbl_colblk_writer_rows(self._w))

    def size(self, rows: Optional[int] = None) -> int:
        return int(self._lib.pbl_colblk_writer_size(self._w, self.rows() if rows is None else rows))

    def finish(self, rows: Optional[int] = None) -> bytes:
        r = self.rows() if rows is None else rows
        n = self.size(r)
        buf = ctypes.create_string_buffer(n)
        m = self._lib.pbl_colblk_writer_finish(self._w, r, buf, n)
        if m != n:
            raise ValueError(f"finish({r}) failed")
        return buf.raw[:n]


def gen_col_blocks(seed: int, n_blocks: int, block_size: int = 32768, schema: int = SCHEMA_CRDB1,
                   alphabet_len: int = 26, roach_key_len: int = 12, prefix_len_shared: int = 4,
                   avg_keys_per_prefix: int = 1, pct_logical: int = 0, value_len: int = 128,
                   base_wall_time: int = 1_700_000_000_000_000_000, n_threads: int = 0,
                   obsolete_every: int = 0, tiering: int = 0, first_block: int = 0):
    """Seeded synthetic colblk blocks at a fixed `block_size` stride (host numpy).
    Defaults are BASELINE config 3: cockroachkvs_bench_test.go:83-89 KeyGenConfig
    (alphabet 26, RoachKeyLen 12, PrefixLenShared 4, 1 key per prefix) with 128 B values.
    `tiering` > 0: Pebblev8 blocks with tiering columns and per-row KVMeta
    (span ids 1..tiering; include/pebble_amd.h pbl_colgen_config).  Block i is
    global block first_block + i of the seed's batch (a rank's shard)."""
    import os
    cfg = N.ColGenConfigC(seed, alphabet_len, prefix_len_shared, roach_key_len, avg_keys_per_prefix,
                          base_wall_time, pct_logical, value_len, obsolete_every, tiering, first_block, 0)
    buf = np.zeros(n_blocks * block_size + 16, np.uint8)
    off = np.empty(n_blocks, np.uint64)
    lens = np.empty(n_blocks, np.uint32)
    nt = n_threads or min(16, os.cpu_count() or 1)
    n = N.gen_lib().pbl_gen_col_blocks(ctypes.byref(cfg), schema, n_blocks, block_size, buf.ctypes.data,
                                   off.ctypes.data, lens.ctypes.data, nt)
    return buf, off, lens, int(n)


def NewDataBlockIter(block: bytes, schema: int = SCHEMA_CRDB1, cmp=bytes_compare,
                     transforms: Transforms = Transforms(), device: str = "cuda") -> Iter:
    """Decode one colblk data block on the device and iterate it."""
    from .batch import BlockBatch, decode
    out = decode(BlockBatch.from_blocks([block], device=device, fmt=schema))
    h = out.to_host()
    st = int(h["blk_status"][0])
    if st == N.PBL_CORRUPT_COLBLK_HEADER:
        raise CorruptionError("pebble: error initializing data block metadata")
    if st != N.PBL_OK:
        raise CorruptionError(f"pebble: corrupt data block ({N.STATUS_NAMES.get(st, st)})")
    return Iter(kvs_of_block(h, 0), cmp, transforms)
