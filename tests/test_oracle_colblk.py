"""Pin the colblk CPU oracle (oracle/colblk_oracle.c) and the native colblk
encoder (pebble_amd/csrc/colblk_writer.cpp) to the reference's own data-block
hex dumps (tests/golden/colblk_golden.json).  CPU only."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, random_rows
from pebble_amd import _native as N
from pebble_amd.colblk import (SCHEMA_CRDB1, SCHEMA_DEFAULT, VALUE_BLOB_HANDLE, VALUE_BLOCK_HANDLE,
                               DataBlockEncoder, gen_col_blocks)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "colblk_golden.json")


@pytest.fixture(scope="module")
def colgolden():
    with open(GOLDEN) as f:
        return json.load(f)


def _schema(c):
    return SCHEMA_CRDB1 if c["schema"] == "crdb1" else SCHEMA_DEFAULT


def _expected(c):
    out = []
    for i, r in enumerate(c["rows"]):
        fl = (N.PBL_KV_PREFIX_CHANGED if r["prefix_changed"] else 0) | (N.PBL_KV_OBSOLETE if r["obsolete"] else 0)
        if r["external"]:
            fl |= N.PBL_KV_VALBLK_HANDLE if (r["vp"] & 0xC0) == 0x80 else N.PBL_KV_BLOB_HANDLE
        out.append((bytes.fromhex(r["key"]), r["trailer"], bytes.fromhex(r["value"]), fl, i))
    return out


def test_fixture_inventory(colgolden):
    names = {c["name"].split(":")[0] for c in colgolden["data_blocks"]}
    # every data-block hex dump the reference's tests print is covered
    assert {"simple", "external_value", "bundle_search", "next_prefix", "finish_without_final_row",
            "rewrite_suffixes", "block_encoding"} <= names
    assert any(c["schema"] == "crdb1" for c in colgolden["data_blocks"])


def test_oracle_decodes_reference_blocks(colgolden):
    """DataBlockIter.First/Next over each reference block yields the KVs the
    reference test wrote (data_block_test.go:76-109; cockroachkvs block_encoding `keys`)."""
    for c in colgolden["data_blocks"]:
        st, kvs = oracle.colblk_decode_block(bytes.fromhex(c["block"]), _schema(c))
        assert st == 0, c["name"]
        assert kvs == _expected(c), c["name"]


def test_writer_reproduces_reference_bytes(colgolden):
    """DataBlockEncoder restatement is byte-exact (incl. Finish(rows-1))."""
    n = 0
    for c in colgolden["data_blocks"]:
        if not c["encoder_exact"]:
            continue
        w = DataBlockEncoder(_schema(c), c["bundle_size"])
        for r in c["writer_rows"]:
            vk = 0 if r["vp"] < 0 else (VALUE_BLOCK_HANDLE if (r["vp"] & 0xC0) == 0x80 else VALUE_BLOB_HANDLE)
            w.add(bytes.fromhex(r["key"]), r["trailer"], bytes.fromhex(r["raw_value"]), vk, r["obsolete"])
        assert w.finish(c["finish_rows"]).hex() == c["block"], c["name"]
        n += 1
    assert n >= 11


@pytest.mark.parametrize("schema", [SCHEMA_DEFAULT, SCHEMA_CRDB1])
@pytest.mark.parametrize("bundle", [1, 4, 16, 64])
def test_writer_oracle_roundtrip(schema, bundle):
    rng = random.Random(1000 * schema + bundle)
    for n in [1, 2, 7, 8, 9, 63, 64, 65, 200, 257, 600]:
        rows = random_rows(rng, schema, n, shared=rng.choice([0, 3, 9]))
        blk, exp = build_block(schema, rows, bundle)
        st, kvs = oracle.colblk_decode_block(blk, schema)
        assert st == 0 and kvs == exp, (schema, bundle, n)


def test_writer_finish_without_final_row():
    """Finish(rows-1) decodes to the first rows-1 KVs (the sstable writer's
    block-overflow path, data_block.go:760-790)."""
    rng = random.Random(5)
    for schema in (SCHEMA_DEFAULT, SCHEMA_CRDB1):
        rows = random_rows(rng, schema, 40)
        w = DataBlockEncoder(schema)
        for r in rows:
            w.add(*r)
        blk_all = w.finish(len(rows) - 1)
        st, kvs = oracle.colblk_decode_block(blk_all, schema)
        _, exp = build_block(schema, rows[:-1])
        assert st == 0 and [k[:3] for k in kvs] == [e[:3] for e in exp]


def test_oracle_corruption():
    rng = random.Random(9)
    rows = random_rows(rng, SCHEMA_CRDB1, 50)
    blk, _ = build_block(SCHEMA_CRDB1, rows)
    assert oracle.colblk_decode_block(blk[:10], SCHEMA_CRDB1)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    bad = bytearray(blk)
    bad[5 + 7] = 3  # column 0 claims type bytes, not prefixbytes
    assert oracle.colblk_decode_block(bytes(bad), SCHEMA_CRDB1)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    zero_rows = bytearray(blk)
    zero_rows[5 + 3:5 + 7] = b"\x00\x00\x00\x00"
    assert oracle.colblk_decode_block(bytes(zero_rows), SCHEMA_CRDB1)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    # the wrong schema is a header error too (crdb1 block read as default)
    assert oracle.colblk_decode_block(blk, SCHEMA_DEFAULT)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    statuses = set()
    for i in range(400):
        b = bytearray(blk)
        for _ in range(rng.randint(1, 4)):
            b[rng.randrange(len(b))] = rng.randrange(256)
        st, kvs = oracle.colblk_decode_block(bytes(b), SCHEMA_CRDB1)
        statuses.add(st)
        assert st in (0, N.PBL_CORRUPT_BOUNDS, N.PBL_CORRUPT_COLBLK_HEADER, N.PBL_UNSUPPORTED)
    assert 0 in statuses and N.PBL_CORRUPT_COLBLK_HEADER in statuses


def test_gen_col_blocks_config3():
    buf, off, lens, n = gen_col_blocks(3, 64)
    assert np.all(lens <= 32768) and np.all(lens > 30000)
    assert np.all(off == np.arange(64, dtype=np.uint64) * 32768)
    r = oracle.decode_batch(buf, off, lens, SCHEMA_CRDB1)
    assert r["status_mask"] == 0 and r["n_kv"] == n
    kl = np.diff(r["key_off"].astype(np.int64))
    assert 190 <= n / 64 <= 240
    # RoachKeyLen 12 + sentinel + 8-byte wall + length byte
    assert r["key_bytes_total"] == 22 * n
    assert r["val_bytes_total"] == 128 * n


def test_mixed_batch_oracle():
    rb, ro, rl, rn = __import__("pebble_amd.rowblk", fromlist=["gen_row_blocks"]).gen_row_blocks(4, 3, 4096)
    cb, co, cl, cn = gen_col_blocks(4, 3, 8192)
    buf = np.concatenate([rb[:3 * 4096], cb[:3 * 8192]])
    off = np.concatenate([ro, co + 3 * 4096]).astype(np.uint64)
    lens = np.concatenate([rl, cl]).astype(np.uint32)
    fmt = np.array([0, 0, 0, 2, 2, 2], np.uint8)
    r = oracle.decode_batch(buf, off, lens, 0, fmt)
    assert r["status_mask"] == 0 and r["n_kv"] == rn + cn


def test_colblk_scan_checksum_matches_decode():
    """The iterate-only CPU baseline (SetNext-shaped scan) sees the same KVs as
    the oracle's full decode."""
    M = (1 << 64) - 1
    for schema in (SCHEMA_DEFAULT, SCHEMA_CRDB1):
        rng = random.Random(40 + schema)
        for n in (1, 17, 300):
            rows = random_rows(rng, schema, n, shared=3)
            blk, exp = build_block(schema, rows, rng.choice([1, 4, 16]))
            buf = np.frombuffer(blk + bytes(16), np.uint8).copy()
            h, cnt = oracle.colblk_scan_checksum(buf, np.array([0], np.uint64), np.array([len(blk)], np.uint32),
                                                 schema)
            st, kvs = oracle.colblk_decode_block(blk, schema)
            x = 1469598103934665603
            for k, tr, v, fl, _ in kvs:
                raw = bytes([v[0]]) if v else b"\0"
                x = ((x ^ tr ^ (k[-1] if k else 0) ^ raw[0] ^ len(v)) * 1099511628211) & M
            assert cnt == n and h == x
