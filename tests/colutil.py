"""Random colblk block construction for the oracle and GPU parity tests.

Blocks are produced by the native restatement of colblk.DataBlockEncoder (pinned
byte-exact to the reference by tests/test_oracle_colblk.py); the expected decode
of each row is derived from the writer input alone (expected_key below), never
from the decoder under test.
"""
import random
import struct

from pebble_amd.colblk import (SCHEMA_CRDB1, SCHEMA_DEFAULT, VALUE_BLOB_HANDLE, VALUE_BLOCK_HANDLE,
                               VALUE_IN_PLACE, DataBlockEncoder)
from pebble_amd import _native as N

KINDS = [0, 1, 1, 1, 2, 7, 18, 23]


def crdb_version(rng: random.Random) -> bytes:
    """A random cockroachkvs version suffix (cockroachkvs.go:140-197 encodings)."""
    r = rng.random()
    if r < 0.10:
        return b""
    if r < 0.15:
        return bytes(8) + b"\x09"  # zero wall time, MVCC-encoded
    wall = rng.getrandbits(64) if rng.random() < 0.5 else rng.randrange(1, 1 << 40)
    if r < 0.55:
        return struct.pack(">Q", wall) + b"\x09"
    if r < 0.75:
        return struct.pack(">QI", wall, rng.getrandbits(32)) + b"\x0d"
    if r < 0.82:
        return struct.pack(">QIB", wall, rng.getrandbits(32), 1) + b"\x0e"  # synthetic bit
    if r < 0.86:
        return bytes(12) + b"\x0d"  # zero wall + zero logical
    n = rng.choice([1, 2, 5, 16, 17, 20])  # untyped (e.g. lock table) versions
    return bytes(rng.getrandbits(8) for _ in range(n)) + bytes([n + 1])


def expected_key(schema: int, key: bytes) -> bytes:
    """The user key MaterializeUserKey returns for a written key
    (cockroachkvs.go:1009-1071: MVCC versions are re-encoded, an all-zero one
    vanishes, the synthetic-bit byte is dropped)."""
    if schema != SCHEMA_CRDB1:
        return key
    vlen = key[-1]
    pl = len(key) - vlen
    roach, ver = key[:pl], key[pl:-1] if vlen else b""
    if vlen in (9, 13, 14):
        wall = int.from_bytes(ver[:8], "big")
        logical = int.from_bytes(ver[8:12], "big") if vlen >= 13 else 0
        if wall == 0 and logical == 0:
            return roach
        if logical == 0:
            return roach + ver[:8] + b"\x09"
        return roach + ver[:12] + b"\x0d"
    return key


def random_rows(rng: random.Random, schema: int, n: int, key_len=(1, 24), shared=0, dup_prob=0.15,
                ext_prob=0.1, val_len=(0, 40)):
    """Sorted random KVs for one block: (key, trailer, value, value_kind, obsolete)."""
    prefix = bytes(rng.choice(b"abcdefgh") for _ in range(shared))
    roots = set()
    while len(roots) < n:
        k = prefix + bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(*key_len)))
        roots.add(k)
    roots = sorted(roots)
    keys = []
    for r in roots:
        reps = 1 + (rng.random() < dup_prob) * rng.randint(1, 5)
        for _ in range(reps):
            if schema == SCHEMA_CRDB1:
                keys.append(r + b"\x00" + crdb_version(rng))
            else:
                suf = b"" if rng.random() < 0.2 else b"@" + str(rng.randint(0, 999)).encode()
                keys.append(r + suf)
            if len(keys) >= n:
                break
        if len(keys) >= n:
            break
    if schema == SCHEMA_CRDB1:
        # sort by roach key, keep version order stable (the writer does not check it)
        keys.sort(key=lambda k: k[: len(k) - k[-1]])
    else:
        keys.sort()
    rows = []
    prev = None
    for i, k in enumerate(keys):
        kind = rng.choice(KINDS)
        vk = VALUE_IN_PLACE
        if rng.random() < ext_prob:
            vk = rng.choice([VALUE_BLOCK_HANDLE, VALUE_BLOB_HANDLE])
        v = bytes(rng.getrandbits(8) for _ in range(rng.randint(*val_len)))
        obs = prev == k or rng.random() < 0.05
        rows.append((k, (rng.randrange(1 << 20) << 8) | kind, v, vk, obs))
        prev = k
    return rows


def build_block(schema: int, rows, bundle: int = 16):
    """Encode rows; returns (block bytes, expected decode list of
    (key, trailer, value, flags, row))."""
    w = DataBlockEncoder(schema, bundle)
    exp = []
    for i, (k, tr, v, vk, obs) in enumerate(rows):
        pe = w.add(k, tr, v, vk, obs)
        fl = 0 if pe else N.PBL_KV_PREFIX_CHANGED
        if obs:
            fl |= N.PBL_KV_OBSOLETE
        val = v
        if vk != VALUE_IN_PLACE:
            vp = (0x80 if vk == VALUE_BLOCK_HANDLE else 0x40) | (0x20 if pe else 0)
            val = bytes([vp]) + v
            fl |= N.PBL_KV_VALBLK_HANDLE if vk == VALUE_BLOCK_HANDLE else N.PBL_KV_BLOB_HANDLE
        exp.append((expected_key(schema, k), tr, val, fl, i))
    return w.finish(), exp


# ---- raw DefaultKeySchema data-block assembly (per-codec embedding) ----------------
# Layout (sstable/colblk/block.go:10-56, data_block.go:600-833): maximum key length
# LE32 (DataBlockCustomHeaderSize), version 1, 7 columns LE16, rows LE32, then per
# column {type u8, page offset LE32}, the pages, one 0x00 pad byte.  Columns of
# colblk.DefaultKeySchema: prefix (PrefixBytes), suffix (RawBytes), trailers (Uint),
# prefixChanged (Bitmap), values (RawBytes), isValueExternal (Bitmap), isObsolete (Bitmap).
DEFAULT_COL_TYPES = [4, 3, 2, 1, 3, 1, 1]
COL_PREFIX, COL_SUFFIX, COL_TRAILERS, COL_PREFIX_CHANGED, COL_VALUES, COL_EXTERNAL, COL_OBSOLETE = range(7)


def _suffix_column(rows: int, tail: int) -> bytes:
    """RawBytes of `rows` slices, all empty but the last (`tail` bytes of 'z')."""
    if tail == 0:
        return b"\x00"  # offsets all zero: uint zero encoding, no data
    assert tail < 256
    return bytes([1]) + bytes(rows) + bytes([tail]) + b"z" * tail


def default_columns(rows: int) -> list:
    """Minimal valid columns for `rows` rows: empty keys and values, zero
    trailers, zero bitmaps."""
    return [bytes([4, 0]),  # PrefixBytes, bundle shift 4, RawBytes offsets all zero
            b"\x00", b"\x00", b"\x01", b"\x00", b"\x01", b"\x01"]


def assemble_block(cols: list, rows: int, max_key_len: int) -> bytes:
    hdr = 4 + 7 + 5 * len(cols)
    offs, pos = [], hdr
    for c in cols:
        offs.append(pos)
        pos += len(c)
    out = bytearray(max_key_len.to_bytes(4, "little") + bytes([1]) + len(cols).to_bytes(2, "little")
                    + rows.to_bytes(4, "little"))
    for t, o in zip(DEFAULT_COL_TYPES, offs):
        out += bytes([t]) + o.to_bytes(4, "little")
    for c in cols:
        out += c
    return bytes(out + b"\x00")


def embed_column(col: int, col_bytes: bytes, col_offset: int, rows: int, max_key_len: int = 0) -> bytes:
    """A DefaultKeySchema block whose column `col` is `col_bytes` (a column the
    reference's codec tests printed, `col_offset` = its start in those bytes'
    buffer), placed at a block offset congruent to it mod 8 so that its
    internal alignment padding stays valid (the suffix column's last slice
    absorbs the shift; col_bytes must come after it)."""
    assert col > COL_SUFFIX or col == COL_PREFIX
    cols = default_columns(rows)
    cols[col] = col_bytes
    for tail in range(0, 9):
        cols[COL_SUFFIX] = _suffix_column(rows, tail)
        start = 4 + 7 + 5 * len(cols) + sum(len(c) for c in cols[:col])
        if col == COL_PREFIX or start % 8 == col_offset % 8:
            return assemble_block(cols, rows, max(max_key_len, tail))
    raise AssertionError("unreachable")


# ---- Pebblev8 tiering columns ------------------------------------------------------
def random_metas(rng: random.Random, n: int):
    """Random base.KVMeta per row (span, attribute), widths 0..8 bytes; about a
    fifth unset (attribute 0: KVMeta.IsSet false, internal/base/internal.go:700)."""
    out = []
    big = rng.choice([1, 300, 70000, 1 << 40])
    for _ in range(n):
        if rng.random() < 0.2:
            out.append((rng.randrange(big), 0))
        else:
            out.append((rng.randrange(big), 1 + rng.randrange(big)))
    return out


def build_block_meta(schema: int, rows, metas, bundle: int = 16, handles=None):
    """A Pebblev8 block (tiering columns): returns (block bytes, expected decode
    as build_block, expected KVMeta per row).  The writer stores a meta only
    when its attribute is set (data_block.go:753-757), so an unset one reads
    back as KVMeta{} whatever its span."""
    w = DataBlockEncoder(schema, bundle, tiering=True)
    exp = []
    for i, ((k, tr, v, vk, obs), m) in enumerate(zip(rows, metas)):
        h = handles[i] if handles else b""
        pe = w.add(k, tr, v, vk, obs, meta=m, secondary_handle=h)
        fl = 0 if pe else N.PBL_KV_PREFIX_CHANGED
        if obs:
            fl |= N.PBL_KV_OBSOLETE
        val = v
        if vk != VALUE_IN_PLACE:
            vp = (0x80 if vk == VALUE_BLOCK_HANDLE else 0x40) | (0x20 if pe else 0)
            val = bytes([vp]) + v
            fl |= N.PBL_KV_VALBLK_HANDLE if vk == VALUE_BLOCK_HANDLE else N.PBL_KV_BLOB_HANDLE
        exp.append((expected_key(schema, k), tr, val, fl, i))
    return w.finish(), exp, [m if m[1] else (0, 0) for m in metas]
