"""ctypes binding of the C-ABI in include/pebble_amd.h (libpebble_amd.so).

The shared library is built in-tree by pebble_amd.build (hipcc, gfx950) and is
the only implementation of the decode path: there is no CPU fallback.  Loading
fails loudly when the library is missing.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PBL_LIB selects the diagnostic (phase-stamp) build for scripts/pipe_stamps.py
LIB_PATH = os.environ.get("PBL_LIB") or os.path.join(_HERE, "libpebble_amd.so")

# status codes (include/pebble_amd.h)
PBL_OK = 0
PBL_CORRUPT_NO_RESTARTS = 1
PBL_CORRUPT_FIRST_KEY = 2
PBL_CORRUPT_BOUNDS = 3
PBL_CORRUPT_COLBLK_HEADER = 4
PBL_UNSUPPORTED = 5
PBL_OVERFLOW = 6
PBL_INVALID_ARG = 7
PBL_DEVICE_ERROR = 8
PBL_TIMEOUT = 9
PBL_CORRUPT_CHECKSUM = 10
PBL_CORRUPT_COMPRESSION = 11
PBL_CORRUPT_FOOTER = 12
PBL_CORRUPT_INDEX = 13
PBL_CORRUPT_VALUE_HANDLE = 14
STATUS_NAMES = {
    0: "OK", 1: "CORRUPT_NO_RESTARTS", 2: "CORRUPT_FIRST_KEY", 3: "CORRUPT_BOUNDS",
    4: "CORRUPT_COLBLK_HEADER", 5: "UNSUPPORTED", 6: "OVERFLOW", 7: "INVALID_ARG",
    8: "DEVICE_ERROR", 9: "TIMEOUT", 10: "CORRUPT_CHECKSUM", 11: "CORRUPT_COMPRESSION",
    12: "CORRUPT_FOOTER", 13: "CORRUPT_INDEX", 14: "CORRUPT_VALUE_HANDLE",
}
# TableFormat (footer magic, version)
PBL_TABLE_LEVELDB, PBL_TABLE_ROCKSDBV2 = 1, 2
PBL_TABLE_PEBBLEV1 = 3  # .. PBL_TABLE_PEBBLEV8 = 10
PBL_TABLE_PEBBLEV5, PBL_TABLE_PEBBLEV6, PBL_TABLE_PEBBLEV7 = 7, 8, 9
PBL_CHECKSUM_NONE, PBL_CHECKSUM_CRC32C, PBL_CHECKSUM_XXHASH, PBL_CHECKSUM_XXHASH64 = 0, 1, 2, 3
PBL_COMPRESSION_NONE, PBL_COMPRESSION_SNAPPY, PBL_COMPRESSION_ZSTD, PBL_COMPRESSION_MINLZ = 0, 1, 7, 8

ABI_VERSION = 8  # include/pebble_amd.h PBL_ABI_VERSION

PBL_FMT_ROW = 0
PBL_FMT_COL_DEFAULT = 1
PBL_FMT_COL_CRDB1 = 2

PBL_ROW_VALUE_PREFIX = 0x1
PBL_ROW_NO_VALUER = 0x2
PBL_ROW_RAW_KEYS = 0x4
PBL_BATCH_VARLEN = 0x100
PBL_ROW_HIDE_OBSOLETE = 0x8
PBL_COL_TIERING = 0x10
PBL_KERNEL_SINGLE = 0x200
PBL_KERNEL_PIPE = 0x400
PBL_KERNEL_POOL = 0x4000
PBL_PHYS_MINLZ_NATIVE = 0x1

PBL_KV_RESTART = 0x01
PBL_KV_RESTART_SAMEPFX = 0x02
PBL_KV_OBSOLETE = 0x04
PBL_KV_INVALID_KEY = 0x08
PBL_KV_VALBLK_HANDLE = 0x10
PBL_KV_BLOB_HANDLE = 0x20
PBL_KV_PREFIX_CHANGED = 0x40

_vp = ctypes.c_void_p
_u8p = ctypes.POINTER(ctypes.c_uint8)


class BlockBatchC(ctypes.Structure):
    _fields_ = [
        ("blocks", _vp), ("block_off", _vp), ("block_len", _vp),
        ("n_blocks", ctypes.c_uint32), ("format", ctypes.c_uint32),
        ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
        ("block_format", _vp), ("synthetic_seq_num", ctypes.c_uint64),
    ]


class ColGenConfigC(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64), ("alphabet_len", ctypes.c_uint32),
        ("prefix_len_shared", ctypes.c_uint32), ("roach_key_len", ctypes.c_uint32),
        ("avg_keys_per_prefix", ctypes.c_uint32), ("base_wall_time", ctypes.c_uint64),
        ("pct_logical", ctypes.c_uint32), ("value_len", ctypes.c_uint32),
        ("obsolete_every", ctypes.c_uint32), ("tiering", ctypes.c_uint32),
        ("first_block", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
    ]


class ZipfConfigC(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64), ("key_min", ctypes.c_uint32), ("key_max", ctypes.c_uint32),
        ("val_min", ctypes.c_uint32), ("val_max", ctypes.c_uint32), ("s", ctypes.c_double),
        ("block_size", ctypes.c_uint32), ("restart_interval", ctypes.c_int32),
        ("first_block", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
    ]


class TotalsC(ctypes.Structure):
    _fields_ = [
        ("n_kv", ctypes.c_uint64), ("key_bytes", ctypes.c_uint64),
        ("val_bytes", ctypes.c_uint64), ("n_restarts", ctypes.c_uint64),
        ("status_mask", ctypes.c_uint32), ("n_bad_blocks", ctypes.c_uint32),
        ("n_slow_blocks", ctypes.c_uint32), ("pad", ctypes.c_uint32),
    ]


class DecodeOutC(ctypes.Structure):
    _fields_ = [
        ("trailer", _vp), ("kv_flags", _vp), ("entry_off", _vp),
        ("key_off", _vp), ("val_off", _vp), ("key_bytes", _vp), ("val_bytes", _vp),
        ("restarts", _vp), ("blk_kv_base", _vp), ("blk_key_base", _vp),
        ("blk_val_base", _vp), ("blk_rst_base", _vp), ("blk_status", _vp),
        ("totals", _vp),
        ("kv_cap", ctypes.c_uint64), ("key_cap", ctypes.c_uint64),
        ("val_cap", ctypes.c_uint64), ("rst_cap", ctypes.c_uint64),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_uint64),
        ("tiering_span_id", _vp), ("tiering_attr", _vp),
    ]


PBL_SPLIT_WHOLE, PBL_SPLIT_TESTKEYS, PBL_SPLIT_CRDB = 0, 1, 2


class PhysBatchC(ctypes.Structure):
    _fields_ = [("bytes", _vp), ("block_off", _vp), ("block_len", _vp), ("n_blocks", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class FooterC(ctypes.Structure):
    _fields_ = [
        ("table_format", ctypes.c_uint32), ("checksum_type", ctypes.c_uint32),
        ("metaindex_off", ctypes.c_uint64), ("metaindex_len", ctypes.c_uint64),
        ("index_off", ctypes.c_uint64), ("index_len", ctypes.c_uint64),
        ("footer_off", ctypes.c_uint64), ("footer_len", ctypes.c_uint64),
        ("attributes", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
    ]


class IndexOutC(ctypes.Structure):
    _fields_ = [("handle_off", _vp), ("handle_len", _vp), ("props_off", _vp), ("props_len", _vp),
                ("blk_base", _vp), ("blk_status", _vp), ("cap", ctypes.c_uint64)]


class KvOutC(ctypes.Structure):
    _fields_ = [("key_off", _vp), ("key_len", _vp), ("val_off", _vp), ("val_len", _vp), ("blk_base", _vp),
                ("blk_status", _vp), ("cap", ctypes.c_uint64)]


class ValueOutC(ctypes.Structure):
    _fields_ = [("val_off", _vp), ("val_bytes", _vp), ("blk_val_base", _vp), ("blk_status", _vp),
                ("val_cap", ctypes.c_uint64)]


class TransformsC(ctypes.Structure):
    _fields_ = [
        ("synthetic_seq_num", ctypes.c_uint64), ("hide_obsolete_points", ctypes.c_uint32),
        ("split", ctypes.c_uint32), ("prefix", _vp), ("suffix", _vp),
        ("prefix_len", ctypes.c_uint32), ("suffix_len", ctypes.c_uint32),
        ("blocks", ctypes.POINTER(BlockBatchC)),
    ]


class KvC(ctypes.Structure):  # pbl_kv (base.InternalKV over the decoded arrays)
    _fields_ = [("user_key", _vp), ("user_key_len", ctypes.c_uint64), ("trailer", ctypes.c_uint64),
                ("value", _vp), ("value_len", ctypes.c_uint64), ("kv_flags", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class KvMetaC(ctypes.Structure):  # pbl_kv_meta (base.KVMeta)
    _fields_ = [("tiering_span_id", ctypes.c_uint64), ("tiering_attribute", ctypes.c_uint64)]


PBL_CMP_DEFAULT, PBL_CMP_TESTKEYS, PBL_CMP_CRDB = 0, 1, 2
_kvp = ctypes.POINTER(KvC)
_u8p = ctypes.c_char_p

# Every symbol include/pebble_amd.h declares, with its ctypes signature.
SIGNATURES = {
    "pbl_data_iter_new": (_vp, []),
    "pbl_data_iter_free": (None, [_vp]),
    "pbl_data_iter_init": (ctypes.c_int, [_vp, ctypes.POINTER(DecodeOutC), ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32]),
    "pbl_data_iter_first": (_kvp, [_vp]),
    "pbl_data_iter_last": (_kvp, [_vp]),
    "pbl_data_iter_next": (_kvp, [_vp]),
    "pbl_data_iter_prev": (_kvp, [_vp]),
    "pbl_data_iter_seek_ge": (_kvp, [_vp, _u8p, ctypes.c_uint64, ctypes.c_uint32]),
    "pbl_data_iter_seek_lt": (_kvp, [_vp, _u8p, ctypes.c_uint64, ctypes.c_uint32]),
    "pbl_data_iter_seek_prefix_ge": (_kvp, [_vp, _u8p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_int)]),
    "pbl_data_iter_first_with_meta": (_kvp, [_vp, ctypes.POINTER(KvMetaC)]),
    "pbl_data_iter_next_with_meta": (_kvp, [_vp, ctypes.POINTER(KvMetaC)]),
    "pbl_data_iter_seek_ge_with_meta": (_kvp, [_vp, _u8p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.POINTER(KvMetaC)]),
    "pbl_data_iter_next_with_same_prefix": (_kvp, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "pbl_data_iter_next_prefix": (_kvp, [_vp, _u8p, ctypes.c_uint64]),
    "pbl_data_iter_is_lower_bound": (ctypes.c_int, [_vp, _u8p, ctypes.c_uint64]),
    "pbl_data_iter_valid": (ctypes.c_int, [_vp]),
    "pbl_data_iter_kv": (_kvp, [_vp]),
    "pbl_data_iter_invalidate": (None, [_vp]),
    "pbl_data_iter_is_data_invalidated": (ctypes.c_int, [_vp]),
    "pbl_key_compare": (ctypes.c_int, [ctypes.c_uint32, _u8p, ctypes.c_uint64, _u8p, ctypes.c_uint64]),
    "pbl_key_split": (ctypes.c_uint64, [ctypes.c_uint32, _u8p, ctypes.c_uint64]),
    "pbl_abi_version": (ctypes.c_int, []),
    "pbl_workspace_bytes": (ctypes.c_uint64, [ctypes.c_uint32]),
    "pbl_decode_batch": (ctypes.c_int, [ctypes.POINTER(BlockBatchC), ctypes.POINTER(DecodeOutC), _vp]),
    "pbl_size_batch": (ctypes.c_int, [ctypes.POINTER(BlockBatchC), ctypes.POINTER(DecodeOutC), _vp]),
    "pbl_struct_layout": (ctypes.c_size_t, [_vp, ctypes.c_size_t]),
    "pbl_transform_workspace_bytes": (ctypes.c_uint64, [ctypes.c_uint32]),
    "pbl_verify_checksums": (ctypes.c_int, [ctypes.POINTER(PhysBatchC), ctypes.c_uint32, _vp, _vp, _vp]),
    "pbl_decompressed_lengths": (ctypes.c_int, [ctypes.POINTER(PhysBatchC), _vp, _vp, _vp]),
    "pbl_decompress_blocks": (ctypes.c_int, [ctypes.POINTER(PhysBatchC), _vp, _vp, _vp, _vp, _vp, _vp]),
    "pbl_parse_footer": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(FooterC)]),
    "pbl_index_handles_row": (ctypes.c_int, [ctypes.POINTER(DecodeOutC), ctypes.c_uint32, ctypes.POINTER(IndexOutC),
                                             _vp]),
    "pbl_index_handles_col": (ctypes.c_int, [ctypes.POINTER(BlockBatchC), ctypes.POINTER(IndexOutC), _vp]),
    "pbl_kv_blocks": (ctypes.c_int, [ctypes.POINTER(BlockBatchC), ctypes.POINTER(KvOutC), _vp]),
    "pbl_valblk_index": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp]),
    "pbl_resolve_values": (ctypes.c_int, [ctypes.POINTER(DecodeOutC), ctypes.c_uint32, ctypes.POINTER(BlockBatchC),
                                          ctypes.POINTER(ValueOutC), _vp]),
    "pbl_transform_batch": (ctypes.c_int, [ctypes.POINTER(DecodeOutC), ctypes.c_uint32, ctypes.POINTER(TransformsC),
                                           ctypes.POINTER(DecodeOutC), _vp]),
    "pbl_rebase_blocks": (ctypes.c_int, [ctypes.POINTER(DecodeOutC), ctypes.c_uint32, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    "pbl_offset_concat": (ctypes.c_int, [ctypes.POINTER(DecodeOutC), ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    "pbl_rowblk_writer_new": (_vp, [ctypes.c_int]),
    "pbl_rowblk_writer_free": (None, [_vp]),
    "pbl_rowblk_writer_reset": (None, [_vp, ctypes.c_int]),
    "pbl_rowblk_writer_add": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64,
                                             ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                             ctypes.c_int64, ctypes.c_int, ctypes.c_uint8, ctypes.c_int]),
    "pbl_rowblk_writer_add_raw": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.c_char_p, ctypes.c_size_t]),
    "pbl_rowblk_writer_estimated_size": (ctypes.c_size_t, [_vp]),
    "pbl_rowblk_writer_entry_count": (ctypes.c_size_t, [_vp]),
    "pbl_rowblk_writer_finish": (ctypes.c_size_t, [_vp, _vp, ctypes.c_size_t]),
    "pbl_gen_row_blocks": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                             _vp, _vp, _vp, ctypes.c_int]),
    "pbl_gen_row_blocks_obs": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                                 ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int]),
    "pbl_colblk_writer_new": (_vp, [ctypes.c_uint32, ctypes.c_int]),
    "pbl_colblk_writer_free": (None, [_vp]),
    "pbl_colblk_writer_reset": (None, [_vp]),
    "pbl_colblk_writer_add": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64,
                                             ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.c_int]),
    "pbl_colblk_writer_set_tiering": (None, [_vp, ctypes.c_int]),
    "pbl_colblk_writer_add_meta": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64,
                                                  ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                                  ctypes.c_size_t]),
    "pbl_colblk_writer_rows": (ctypes.c_uint32, [_vp]),
    "pbl_colblk_writer_size": (ctypes.c_size_t, [_vp, ctypes.c_uint32]),
    "pbl_colblk_writer_finish": (ctypes.c_size_t, [_vp, ctypes.c_uint32, _vp, ctypes.c_size_t]),
    "pbl_gen_col_blocks": (ctypes.c_uint64, [ctypes.POINTER(ColGenConfigC), ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int]),
    "pbl_gen_zipf_blocks": (ctypes.c_uint64, [ctypes.POINTER(ZipfConfigC), ctypes.c_uint32, ctypes.c_uint32,
                                              _vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_int]),
}

_lib = None
_gen_lib = None


def gen_lib() -> ctypes.CDLL:
    """The library for host-only work (synthetic generators, block writers):
    always the in-tree build, so that an A/B run of an older decoder build
    (PBL_LIB) generates exactly the same inputs."""
    global _gen_lib
    if not os.environ.get("PBL_LIB"):
        return lib()
    if _gen_lib is None:
        L = ctypes.CDLL(os.path.join(_HERE, "libpebble_amd.so"))
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _gen_lib = L
    return _gen_lib


def lib() -> ctypes.CDLL:
    """Load libpebble_amd.so (torch is imported first so that the HIP runtime it
    bundles is the one the library binds to: same SONAME, one runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback for the decode path.")
    try:
        import torch  # noqa: F401  (binds libamdhip64.so.7 first)
    except Exception:  # pragma: no cover - torch is always present in this image
        pass
    L = ctypes.CDLL(LIB_PATH)
    ab_build = bool(os.environ.get("PBL_LIB"))
    for name, (res, args) in SIGNATURES.items():
        if ab_build and not hasattr(L, name):
            continue  # an older A/B build (scripts/ab.sh): entry points it predates stay unbound
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.pbl_abi_version() != ABI_VERSION and not ab_build:
        raise RuntimeError("libpebble_amd.so ABI mismatch")
    _lib = L
    return L
