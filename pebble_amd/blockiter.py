"""blockiter.Data over one decoded block (host side).

`DataIter` wraps the library's pbl_data_iter (pebble_amd/csrc/data_iter.cpp):
rowblk.Iter / colblk.DataBlockIter positioning (sstable/blockiter/
block_iter.go:19-108) over the flat arrays of a decoded batch copied to host
memory (`DecodedBatch.to_host()`).  The same C entry points are what the Go cgo
shim of INTEGRATION.md binds.  Positioning methods return an InternalKV or
None, like the Go iterators return *base.InternalKV or nil."""
import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _native as N
from .rowblk import InternalKV


class DataIter:
    def __init__(self, host: dict, block: int, comparer: int = N.PBL_CMP_DEFAULT,
                 hide_obsolete_points: bool = False):
        self._lib = N.lib()
        nb = len(host["blk_status"])
        self._keep = {}  # the arrays the C struct points into
        o = N.DecodeOutC()
        for k in ("trailer", "kv_flags", "key_off", "val_off", "key_bytes", "val_bytes", "blk_kv_base",
                  "blk_key_base", "blk_val_base", "blk_status"):
            a = host[k]
            a = np.ascontiguousarray(a if a is not None and a.size else np.zeros(1, a.dtype if a is not None
                                                                                 else np.uint8))
            self._keep[k] = a
            setattr(o, k, a.ctypes.data)
        for k in ("tiering_span_id", "tiering_attr"):  # KVMeta arrays, when decoded
            a = host.get(k)
            if a is not None:
                a = np.ascontiguousarray(a if a.size else np.zeros(1, np.uint64))
                self._keep[k] = a
                setattr(o, k, a.ctypes.data)
        self._out = o
        self._it = self._lib.pbl_data_iter_new()
        if not self._it:
            raise MemoryError("pbl_data_iter_new")
        self.status = self._lib.pbl_data_iter_init(self._it, ctypes.byref(o), nb, block, comparer,
                                                   1 if hide_obsolete_points else 0)

    def __del__(self):
        if getattr(self, "_it", None):
            self._lib.pbl_data_iter_free(self._it)
            self._it = None

    @staticmethod
    def _kv(p) -> Optional[InternalKV]:
        if not p:
            return None
        k = p.contents
        uk = ctypes.string_at(k.user_key, k.user_key_len) if k.user_key_len else b""
        v = ctypes.string_at(k.value, k.value_len) if k.value_len else b""
        return InternalKV(uk, int(k.trailer), v, int(k.kv_flags))

    def First(self):
        return self._kv(self._lib.pbl_data_iter_first(self._it))

    def Last(self):
        return self._kv(self._lib.pbl_data_iter_last(self._it))

    def Next(self):
        return self._kv(self._lib.pbl_data_iter_next(self._it))

    def Prev(self):
        return self._kv(self._lib.pbl_data_iter_prev(self._it))

    def SeekGE(self, key: bytes, flags: int = 0):
        return self._kv(self._lib.pbl_data_iter_seek_ge(self._it, key, len(key), flags))

    def SeekLT(self, key: bytes, flags: int = 0):
        return self._kv(self._lib.pbl_data_iter_seek_lt(self._it, key, len(key), flags))

    # MetaIterator (colblk data_block.go:1574-1600): (kv, (TieringSpanID, TieringAttribute))
    def _meta(self, p, m) -> Tuple[Optional[InternalKV], Tuple[int, int]]:
        return self._kv(p), (int(m.tiering_span_id), int(m.tiering_attribute))

    def FirstWithMeta(self):
        m = N.KvMetaC()
        return self._meta(self._lib.pbl_data_iter_first_with_meta(self._it, ctypes.byref(m)), m)

    def NextWithMeta(self):
        m = N.KvMetaC()
        return self._meta(self._lib.pbl_data_iter_next_with_meta(self._it, ctypes.byref(m)), m)

    def SeekGEWithMeta(self, key: bytes, flags: int = 0):
        m = N.KvMetaC()
        return self._meta(self._lib.pbl_data_iter_seek_ge_with_meta(self._it, key, len(key), flags,
                                                                   ctypes.byref(m)), m)

    def SeekPrefixGE(self, key: bytes, flags: int = 0) -> Tuple[Optional[InternalKV], bool]:
        miss = ctypes.c_int(0)
        kv = self._kv(self._lib.pbl_data_iter_seek_prefix_ge(self._it, key, len(key), flags, ctypes.byref(miss)))
        return kv, bool(miss.value)

    def NextWithSamePrefix(self) -> Tuple[Optional[InternalKV], bool]:
        ex = ctypes.c_int(0)
        kv = self._kv(self._lib.pbl_data_iter_next_with_same_prefix(self._it, ctypes.byref(ex)))
        return kv, bool(ex.value)

    def NextPrefix(self, succ_key: bytes):
        return self._kv(self._lib.pbl_data_iter_next_prefix(self._it, succ_key, len(succ_key)))

    def IsLowerBound(self, key: bytes) -> bool:
        return bool(self._lib.pbl_data_iter_is_lower_bound(self._it, key, len(key)))

    def Valid(self) -> bool:
        return bool(self._lib.pbl_data_iter_valid(self._it))

    def KV(self):
        return self._kv(self._lib.pbl_data_iter_kv(self._it))

    def Invalidate(self) -> None:
        self._lib.pbl_data_iter_invalidate(self._it)

    def IsDataInvalidated(self) -> bool:
        return bool(self._lib.pbl_data_iter_is_data_invalidated(self._it))

    def Close(self) -> None:
        self.Invalidate()


def key_compare(comparer: int, a: bytes, b: bytes) -> int:
    return N.lib().pbl_key_compare(comparer, a, len(a), b, len(b))


def key_split(comparer: int, key: bytes) -> int:
    return int(N.lib().pbl_key_split(comparer, key, len(key)))
