"""Expected scans of the reference's columnar tables (tests/golden/tables.json,
made by tests/golden/make_table_fixtures.py from tool/testdata/sstable_scan)."""
import json
import os

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "tables.json")) as f:
    TABLES = json.load(f)
KV_VALBLK_HANDLE, KV_BLOB_HANDLE = 0x10, 0x20


def table_bytes(name: str) -> bytes:
    return open(os.path.join(GOLDEN, "sst", name), "rb").read()


def blob_handle(v: bytes):
    """blob.InlineHandle after the value prefix byte (blob/handle.go:104-110):
    [ReferenceID, BlockID, ValueID, ValueLen] as `sstable scan` prints them."""
    ref, a = oracle.go_uvarint(v, 1)
    ln, b = oracle.go_uvarint(v, 1 + a)
    blk, c = oracle.go_uvarint(v, 1 + a + b)
    vid, d = oracle.go_uvarint(v, 1 + a + b + c)
    assert min(a, b, c, d) > 0 and 1 + a + b + c + d == len(v)
    return [ref, blk, vid, ln]


def check_scan(name: str, kvs):
    """kvs = [(user_key, trailer, value, kv_flags)] in table order must print as
    the reference's `sstable scan` lines: key, #seq,KIND, [hex value] or
    [(fREF,blkB,idI,lenL)] with the value a blob handle."""
    exp = TABLES[name]["kvs"]
    assert len(kvs) == len(exp)
    for i, ((k, t, v, fl), e) in enumerate(zip(kvs, exp)):
        assert (k.hex(), t >> 8, t & 0xFF) == (e["key"], e["seq"], e["kind"]), (name, i)
        if e["blob"] is not None:
            assert fl & KV_BLOB_HANDLE and not fl & KV_VALBLK_HANDLE, (name, i)
            assert blob_handle(v) == e["blob"], (name, i)
        else:
            assert not fl & KV_BLOB_HANDLE, (name, i)
            assert v.hex() == e["value"], (name, i)
