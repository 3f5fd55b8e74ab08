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
