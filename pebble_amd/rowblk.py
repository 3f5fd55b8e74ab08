"""Host-side mirror of Pebble's sstable/rowblk API over the device decoder.

  Writer      — rowblk.Writer (sstable/rowblk/rowblk_writer.go:48-320), native
  NewIter     — rowblk.NewIter / Iter.Init (rowblk_iter.go:229-276): the block is
                decoded on the GPU by libpebble_amd.so, the iterator then walks
                the flat decoded arrays
  Iter        — First/Next/Last/Prev/SeekGE/SeekLT with the blockiter.Transforms
                SyntheticSeqNum and HideObsoletePoints (transforms.go:20-56)
  gen_row_blocks — seeded synthetic batches

Errors mirror the reference: a corrupt block raises CorruptionError carrying
the same condition base.CorruptionErrorf reports in rowblk_iter.go:249-251,
471-476.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _native as N

SEQ_NUM_MAX = (1 << 56) - 1
KIND_DELETE, KIND_SET, KIND_MERGE = 0, 1, 2
KIND_INVALID = 191


def make_trailer(seq: int, kind: int) -> int:
    """base.MakeTrailer (internal/base/internal.go:279-281)."""
    return (seq << 8) | kind


class CorruptionError(Exception):
    pass


@dataclass(frozen=True)
class InternalKV:
    user_key: bytes
    trailer: int
    value: bytes
    flags: int = 0

    def seq_num(self) -> int:
        return self.trailer >> 8

    def kind(self) -> int:
        return self.trailer & 0xFF


@dataclass
class Transforms:
    """blockiter.Transforms (sstable/blockiter/transforms.go:20-56).  Iter
    applies synthetic_seq_num and hide_obsolete_points while iterating; a whole
    decoded batch takes all four on the device (pebble_amd.transforms)."""
    synthetic_seq_num: int = 0
    hide_obsolete_points: bool = False
    synthetic_prefix: bytes = b""
    synthetic_suffix: bytes = b""
    split: int = 0  # PBL_SPLIT_*: the comparer's Split (finds the suffix a synthetic suffix replaces)


class Writer:
    """rowblk.Writer backed by the native restatement."""

    def __init__(self, restart_interval: int = 16):
        self._lib = N.gen_lib()
        self._w = self._lib.pbl_rowblk_writer_new(restart_interval)
        self.restart_interval = restart_interval

    def __del__(self):
        w, self._w = getattr(self, "_w", None), None
        if w:
            self._lib.pbl_rowblk_writer_free(w)

    def reset(self, restart_interval: Optional[int] = None):
        self._lib.pbl_rowblk_writer_reset(self._w, restart_interval or self.restart_interval)

    def add(self, user_key: bytes, trailer: int, value: bytes = b"") -> None:
        self.add_with_optional_value_prefix(user_key, trailer, False, value, len(user_key), False, 0, False)

    def add_with_optional_value_prefix(self, user_key: bytes, trailer: int, is_obsolete: bool, value: bytes,
                                       max_shared_key_len: int, add_value_prefix: bool, value_prefix: int,
                                       set_has_same_key_prefix: bool) -> None:
        rc = self._lib.pbl_rowblk_writer_add(self._w, user_key, len(user_key), trailer, int(is_obsolete),
                                             value, len(value), max_shared_key_len, int(add_value_prefix),
                                             value_prefix, int(set_has_same_key_prefix))
        if rc != N.PBL_OK:
            raise ValueError("rowblk: block size exceeds maximum size")

    def add_raw(self, key: bytes, value: bytes = b"") -> None:
        rc = self._lib.pbl_rowblk_writer_add_raw(self._w, key, len(key), value, len(value))
        if rc != N.PBL_OK:
            raise ValueError("rowblk: block size exceeds maximum size")

    def estimated_size(self) -> int:
        return int(self._lib.pbl_rowblk_writer_estimated_size(self._w))

    def entry_count(self) -> int:
        return int(self._lib.pbl_rowblk_writer_entry_count(self._w))

    def finish(self) -> bytes:
        n = self.estimated_size() + 4  # an empty block gains its single restart (:291-299)
        buf = ctypes.create_string_buffer(n)
        m = self._lib.pbl_rowblk_writer_finish(self._w, buf, n)
        assert m <= n, (m, n)
        return buf.raw[:m]


def gen_row_blocks(seed: int, n_blocks: int, block_size: int = 32768, restart_interval: int = 16,
                   key_len: int = 16, val_len: int = 100, value_prefix: bool = False, n_threads: int = 0,
                   obsolete_every: int = 0, first_block: int = 0):
    """Seeded synthetic row blocks at a fixed `block_size` stride (host numpy).
    obsolete_every > 0: the k-th key of a block with k % obsolete_every ==
    obsolete_every - 1 carries the trailer's obsolete bit.  Block i is global
    block first_block + i of the seed's batch (a rank's shard)."""
    buf = np.empty(n_blocks * block_size + 16, np.uint8)
    buf[-16:] = 0
    off = np.empty(n_blocks, np.uint64)
    lens = np.empty(n_blocks, np.uint32)
    n_kv = N.gen_lib().pbl_gen_row_blocks_obs(seed, first_block, n_blocks, block_size, restart_interval, key_len, val_len,
                                          int(value_prefix), obsolete_every, buf.ctypes.data, off.ctypes.data,
                                          lens.ctypes.data, n_threads)
    return buf, off, lens, int(n_kv)


Compare = Callable[[bytes, bytes], int]


def bytes_compare(a: bytes, b: bytes) -> int:
    return (a > b) - (a < b)


class Iter:
    """rowblk.Iter over one block's decoded KVs (positioning semantics of
    rowblk_iter.go First :1061, Next :1145, Last :1099, Prev, SeekGE, SeekLT)."""

    def __init__(self, kvs: Sequence[InternalKV], cmp: Compare = bytes_compare,
                 transforms: Transforms = Transforms()):
        self._kvs = list(kvs)
        self._cmp = cmp
        self._t = transforms
        self._i = -1  # -1: before first; len: after last

    def _hidden(self, i: int) -> bool:
        return self._t.hide_obsolete_points and bool(self._kvs[i].flags & N.PBL_KV_OBSOLETE)

    def _kv(self) -> Optional[InternalKV]:
        if not (0 <= self._i < len(self._kvs)):
            return None
        kv = self._kvs[self._i]
        if self._t.synthetic_seq_num:
            kv = InternalKV(kv.user_key, (self._t.synthetic_seq_num << 8) | (kv.trailer & 0xFF), kv.value, kv.flags)
        return kv

    def _fwd(self, i: int) -> Optional[InternalKV]:
        while i < len(self._kvs) and self._hidden(i):
            i += 1
        self._i = min(i, len(self._kvs))
        return self._kv()

    def _bwd(self, i: int) -> Optional[InternalKV]:
        while i >= 0 and self._hidden(i):
            i -= 1
        self._i = max(i, -1)
        return self._kv()

    def Valid(self) -> bool:
        return 0 <= self._i < len(self._kvs)

    def First(self):
        return self._fwd(0)

    def Last(self):
        return self._bwd(len(self._kvs) - 1)

    def Next(self):
        return self._fwd(self._i + 1) if self._i < len(self._kvs) else None

    def Prev(self):
        return self._bwd(self._i - 1) if self._i >= 0 else None

    def SeekGE(self, key: bytes, flags: int = 0):
        lo, hi = 0, len(self._kvs)
        while lo < hi:
            m = (lo + hi) // 2
            if self._cmp(self._kvs[m].user_key, key) < 0:
                lo = m + 1
            else:
                hi = m
        return self._fwd(lo)

    def SeekLT(self, key: bytes, flags: int = 0):
        lo, hi = 0, len(self._kvs)
        while lo < hi:
            m = (lo + hi) // 2
            if self._cmp(self._kvs[m].user_key, key) < 0:
                lo = m + 1
            else:
                hi = m
        return self._bwd(lo - 1)

    def Close(self):
        self._kvs = []
        return None


def kvs_of_block(decoded: dict, b: int) -> List[InternalKV]:
    """Extract block b's KVs from a host readout (DecodedBatch.to_host())."""
    nb = len(decoded["blk_status"])
    kv0, kv1 = int(decoded["blk_kv_base"][b]), int(decoded["blk_kv_base"][b + 1])
    kb, vb = int(decoded["blk_key_base"][b]), int(decoded["blk_val_base"][b])
    ko, vo = decoded["key_off"], decoded["val_off"]
    keys, vals = decoded["key_bytes"], decoded["val_bytes"]
    out = []
    for j in range(kv1 - kv0):
        o = kv0 + b + j
        k = keys[kb + ko[o]: kb + ko[o + 1]].tobytes()
        v = vals[vb + vo[o]: vb + vo[o + 1]].tobytes()
        out.append(InternalKV(k, int(decoded["trailer"][kv0 + j]), v, int(decoded["kv_flags"][kv0 + j])))
    assert nb >= b
    return out


def NewIter(block: bytes, cmp: Compare = bytes_compare, transforms: Transforms = Transforms(),
            has_value_prefix: bool = False, device: str = "cuda") -> Iter:
    """rowblk.NewIter: decode `block` on the device and return an iterator over it."""
    from .batch import BlockBatch, decode
    flags = N.PBL_ROW_VALUE_PREFIX if has_value_prefix else 0
    out = decode(BlockBatch.from_blocks([block], device=device, flags=flags))
    h = out.to_host()
    st = int(h["blk_status"][0])
    if st == N.PBL_CORRUPT_NO_RESTARTS:
        raise CorruptionError("pebble/table: invalid table (block has no restart points)")
    if st == N.PBL_CORRUPT_FIRST_KEY:
        raise CorruptionError("pebble/table: invalid firstKey in block")
    if st != N.PBL_OK:
        raise CorruptionError(f"pebble/table: corrupt block ({N.STATUS_NAMES.get(st, st)})")
    return Iter(kvs_of_block(h, 0), cmp, transforms)
