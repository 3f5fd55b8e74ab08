"""Pebblev8 tiering metadata on the CPU side: the colblk oracle's decodeMeta
(FLAG_TIERING) and the native encoder's tiering columns, pinned to the only
tiering bytes the reference holds -- the v8 data blocks of
sstable/testdata/writer_tiering_histogram -- and to the KVMeta KATs of
colblk/data_block_meta_test.go:27-33 and sstable/testdata/writer_v8:388-402
(tests/golden/colblk_golden.json "tiering").  Random v8 blocks beyond those are
"parity unpinned" in the sense of DESIGN.md §5: the restatement checked against
itself (writer -> oracle round trips)."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from colutil import build_block, build_block_meta, random_metas, random_rows
from pebble_amd import _native as N
from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT, VALUE_IN_PLACE, DataBlockEncoder

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "colblk_golden.json")
T = oracle.FLAG_TIERING


@pytest.fixture(scope="module")
def tiering():
    with open(GOLDEN) as f:
        return json.load(f)["tiering"]


def _kat_block(kvs, tiering=True):
    """Encode a KAT's (ikey, value, span, attr) list with the testkeys DefaultKeySchema."""
    w = DataBlockEncoder(SCHEMA_DEFAULT, 16, tiering=tiering)
    for ik, v, sp, at in kvs:
        i, j = ik.index("#"), ik.index(",")
        kind = {"SET": 1, "DEL": 0}[ik[j + 1:]]
        w.add(ik[:i].encode(), int(ik[i + 1:j]) << 8 | kind, v.encode(), meta=(sp, at))
    return w.finish()


def test_fixture_inventory(tiering):
    assert len(tiering["blocks"]) == 2 and len(tiering["kats"]) == 2
    b0 = bytes.fromhex(tiering["blocks"][0]["block"])
    assert len(b0) == 268 and b0[5:7] == b"\x0a\x00"  # 10 columns: 2 key + 8 data (dataBlockColumnMaxV2)


def test_oracle_decodes_reference_v8_blocks(tiering):
    """The reference's v8 blocks decode to the KVs its test wrote and, under
    FLAG_TIERING, to the KVMeta its writer stored (NextWithMeta)."""
    for c in tiering["blocks"]:
        blk = bytes.fromhex(c["block"])
        st, kvs = oracle.colblk_decode_block(blk, SCHEMA_DEFAULT, T, meta=True)
        assert st == 0, c["name"]
        assert len(kvs) == len(c["rows"])
        for kv, r in zip(kvs, c["rows"]):
            k, tr, v, fl, _, sp, at = kv
            assert k == bytes.fromhex(r["key"]) and tr == r["trailer"], c["name"]
            assert (sp, at) == (r["span"], r["attr"]), c["name"]
            assert bool(fl & N.PBL_KV_PREFIX_CHANGED) == r["prefix_changed"]
            if r["external"]:
                assert fl & N.PBL_KV_BLOB_HANDLE and v[0] & 0xC0 == 0x40
            else:
                assert v == bytes.fromhex(r["value"])
        # without the tiering config the same KVs, and KVMeta{} (!SupportsTiering)
        st2, kvs2 = oracle.colblk_decode_block(blk, SCHEMA_DEFAULT, 0, meta=True)
        assert st2 == 0 and [x[:5] for x in kvs2] == [x[:5] for x in kvs]
        assert all(x[5:] == (0, 0) for x in kvs2)


def test_writer_reproduces_reference_v8_block(tiering):
    """DataBlockEncoder.Init(WithTieringColumns) restatement is byte-exact on the
    reference's v8 block (span/attribute UintBuilders InitWithDefault, the
    secondary-handle RawBytes column)."""
    n = 0
    for c in tiering["blocks"]:
        if not c["encoder_exact"]:
            continue
        w = DataBlockEncoder(SCHEMA_DEFAULT, c["bundle_size"], tiering=True)
        for r in c["rows"]:
            w.add(bytes.fromhex(r["key"]), r["trailer"], bytes.fromhex(r["value"]), VALUE_IN_PLACE, r["obsolete"],
                  meta=(r["span"], r["attr"]))
        assert w.finish().hex() == c["block"], c["name"]
        n += 1
    assert n == 1


def test_meta_kats(tiering):
    """TestDataBlockIterWithMeta and writer_v8's scan-compaction: encode the KVs
    with their metas, decode with FLAG_TIERING: the metas the reference's
    iterator returned."""
    for kat in tiering["kats"]:
        blk = _kat_block(kat["kvs"])
        st, kvs = oracle.colblk_decode_block(blk, SCHEMA_DEFAULT, T, meta=True)
        assert st == 0, kat["source"]
        assert [(x[5], x[6]) for x in kvs] == [(sp, at) for _, _, sp, at in kat["kvs"]], kat["source"]
        assert [x[2] for x in kvs] == [v.encode() for _, v, _, _ in kat["kvs"]]


@pytest.mark.parametrize("schema", [SCHEMA_DEFAULT, SCHEMA_CRDB1])
def test_v8_roundtrip_random(schema):
    rng = random.Random(77 + schema)
    for n in (1, 2, 9, 64, 65, 300, 1000):
        rows = random_rows(rng, schema, n, shared=rng.choice([0, 4]))
        metas = random_metas(rng, len(rows))
        handles = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 0, 5, 9]))) for _ in rows]
        blk, exp, emeta = build_block_meta(schema, rows, metas, rng.choice([1, 16]), handles)
        st, kvs = oracle.colblk_decode_block(blk, schema, T, meta=True)
        assert st == 0 and [x[:5] for x in kvs] == exp and [x[5:] for x in kvs] == emeta, (schema, n)
        # the key/value decode is the v7 one (the extra columns follow isObsolete)
        blk7, exp7 = build_block(schema, rows)
        assert oracle.colblk_decode_block(blk7, schema)[1] == exp7 == exp


def test_tiering_flag_on_v7_block_and_corrupt_columns():
    """initTieringMetadata panics (Go) when the columns are missing or malformed:
    CORRUPT_COLBLK_HEADER; the key/value decode without the flag is unaffected."""
    rng = random.Random(3)
    rows = random_rows(rng, SCHEMA_DEFAULT, 40)
    blk7, _ = build_block(SCHEMA_DEFAULT, rows)
    assert oracle.colblk_decode_block(blk7, SCHEMA_DEFAULT, T)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    assert oracle.colblk_decode_block(blk7, SCHEMA_DEFAULT, 0)[0] == 0
    blk, _, _ = build_block_meta(SCHEMA_DEFAULT, rows, random_metas(rng, 40))
    nsc = 2
    h_span = 4 + 7 + 5 * (nsc + 5)  # directory entry of the span column
    bad = bytearray(blk)
    bad[h_span] = 3  # span column claims RawBytes
    assert oracle.colblk_decode_block(bytes(bad), SCHEMA_DEFAULT, T)[0] == N.PBL_CORRUPT_COLBLK_HEADER
    assert oracle.colblk_decode_block(bytes(bad), SCHEMA_DEFAULT, 0)[0] == 0
    bad = bytearray(blk)
    s = int.from_bytes(blk[h_span + 1:h_span + 5], "little")
    bad[s] = 0x03  # invalid Uint encoding (width 3)
    assert oracle.colblk_decode_block(bytes(bad), SCHEMA_DEFAULT, T)[0] == N.PBL_CORRUPT_COLBLK_HEADER


def test_batch_meta_layout_mixed():
    """orc_decode_batch with meta: colblk KVs carry their metas, row KVs
    KVMeta{} (rowblk.Iter has no meta columns)."""
    from pebble_amd.rowblk import gen_row_blocks
    rng = random.Random(11)
    rb, ro, rl, rn = gen_row_blocks(4, 2, 4096)
    blocks, metas = [], []
    for _ in range(3):
        rows = random_rows(rng, SCHEMA_CRDB1, rng.randint(5, 80))
        m = random_metas(rng, len(rows))
        blk, _, em = build_block_meta(SCHEMA_CRDB1, rows, m)
        blocks.append(blk)
        metas.append(em)
    row = [rb[int(ro[i]):int(ro[i]) + int(rl[i])].tobytes() for i in range(2)]
    parts = [row[0], blocks[0], blocks[1], row[1], blocks[2]]
    fmt = np.array([0, 2, 2, 0, 2], np.uint8)
    offs, pos = [], 0
    for p in parts:
        pos = (pos + 7) // 8 * 8
        offs.append(pos)
        pos += len(p)
    buf = np.zeros(pos + 16, np.uint8)
    for o, p in zip(offs, parts):
        buf[o:o + len(p)] = np.frombuffer(p, np.uint8)
    r = oracle.decode_batch(buf, np.array(offs, np.uint64), np.array([len(p) for p in parts], np.uint32), 0, fmt,
                            T, meta=True)
    assert r["status_mask"] == 0
    kvb = r["blk_kv_base"]
    want = {1: metas[0], 2: metas[1], 4: metas[2]}
    for b in range(5):
        sp = r["tiering_span_id"][kvb[b]:kvb[b + 1]]
        at = r["tiering_attr"][kvb[b]:kvb[b + 1]]
        got = list(zip(sp.tolist(), at.tolist()))
        assert got == (want[b] if b in want else [(0, 0)] * len(got)), b
