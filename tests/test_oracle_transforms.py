"""The oracle's restatement of blockiter.Transforms over a decoded batch
(oracle.transform_batch) pinned by the reference's own transform scans:
sstable/colblk/testdata/data_block/transforms (synthetic-seq-num,
hide-obsolete-points, synthetic-prefix, synthetic-suffix; data_block_test.go
140-160), each block re-encoded byte-exactly by the DataBlockEncoder
restatement, decoded by the oracle, transformed, and its forward scan compared
with the `first`/`next` lines the reference printed."""
import json
import os

import numpy as np
import pytest

import oracle
from pebble_amd.colblk import SCHEMA_DEFAULT, VALUE_BLOB_HANDLE, VALUE_BLOCK_HANDLE, DataBlockEncoder

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "colblk_golden.json")
with open(GOLDEN) as f:
    TRANSFORMS = json.load(f)["transforms"]


def encode_rows(rows, bundle=16) -> bytes:
    w = DataBlockEncoder(SCHEMA_DEFAULT, bundle)
    for r in rows:
        vk = 0 if r["vp"] < 0 else (VALUE_BLOCK_HANDLE if (r["vp"] & 0xC0) == 0x80 else VALUE_BLOB_HANDLE)
        w.add(bytes.fromhex(r["key"]), r["trailer"], bytes.fromhex(r["raw_value"]), vk, r["obsolete"])
    return w.finish()


def forward(d: dict, b: int = 0):
    """(user key, trailer, value) of block b's KVs in order."""
    kv0, kv1 = int(d["blk_kv_base"][b]), int(d["blk_kv_base"][b + 1])
    kb, vb = int(d["blk_key_base"][b]), int(d["blk_val_base"][b])
    out = []
    for j in range(kv1 - kv0):
        o = kv0 + b + j
        out.append((d["key_bytes"][kb + int(d["key_off"][o]): kb + int(d["key_off"][o + 1])].tobytes(),
                    int(d["trailer"][kv0 + j]),
                    d["val_bytes"][vb + int(d["val_off"][o]): vb + int(d["val_off"][o + 1])].tobytes()))
    return out


def check_scan(got, exp, ctx):
    n = len([e for e in exp if e is not None])
    for (k, tr, v), e in zip(got, exp[:n]):
        assert k == bytes.fromhex(e[0]), ctx
        assert v == bytes.fromhex(e[3]), ctx
        if e[1] is not None:
            assert (tr >> 8, tr & 0xFF) == (e[1], e[2]), ctx
    if exp and exp[-1] is None:
        assert len(got) == n, ctx  # the reference's iterator was exhausted there
    else:
        assert len(got) >= n, ctx


def cases():
    for t in TRANSFORMS:
        for it in t["iters"]:
            yield pytest.param(t, it, id=f"transforms:{it['line']}")


@pytest.mark.parametrize("t,it", list(cases()))
def test_oracle_transforms_match_reference_scans(t, it):
    blk = encode_rows(t["rows"])
    buf = np.frombuffer(blk + b"\0" * 16, np.uint8).copy()
    d = oracle.decode_batch(buf, np.array([0], np.uint64), np.array([len(blk)], np.uint32), SCHEMA_DEFAULT)
    assert d["status_mask"] == 0
    x = oracle.transform_batch(d, it["seq_num"], it["hide_obsolete"], bytes.fromhex(it["prefix"]),
                               bytes.fromhex(it["suffix"]), split=1)
    check_scan(forward(x), it["forward"], f"{t['source']} iter@{it['line']}")


def test_transform_fixture_inventory():
    its = [it for t in TRANSFORMS for it in t["iters"]]
    assert any(it["seq_num"] for it in its) and any(it["hide_obsolete"] for it in its)
    assert any(it["prefix"] for it in its) and any(it["suffix"] for it in its)


def test_identity_transform_is_identity():
    t = TRANSFORMS[0]
    blk = encode_rows(t["rows"])
    buf = np.frombuffer(blk + b"\0" * 16, np.uint8).copy()
    d = oracle.decode_batch(buf, np.array([0], np.uint64), np.array([len(blk)], np.uint32), SCHEMA_DEFAULT)
    x = oracle.transform_batch(d)
    for k in ("trailer", "kv_flags", "entry_off", "key_off", "val_off", "key_bytes", "val_bytes", "blk_kv_base",
              "blk_key_base", "blk_val_base"):
        assert np.array_equal(x[k], d[k]), k


def test_oracle_seqnum_transform_matches_host_iter(golden):
    """Row blocks: the batch restatement agrees with the host Iter's
    SyntheticSeqNum / HideObsoletePoints (pinned on the GPU by
    test_rowblk_iter_datadriven_on_gpu against rowblk_iter's globalSeqNum cases)."""
    import random
    from test_rowblk_gpu import pack, random_block
    from pebble_amd.rowblk import InternalKV, Iter, Transforms
    rng = random.Random(3)
    blocks = [random_block(rng)[0] for _ in range(30)]
    buf, off, lens = pack(blocks)
    d = oracle.rowblk_decode_batch(buf, off, lens)
    for seq, hide in ((0, True), (77, False), (5, True)):
        x = oracle.transform_batch(d, seq, hide)
        for b in range(len(blocks)):
            if d["blk_status"][b] != 0:
                continue
            kv0, kv1 = int(d["blk_kv_base"][b]), int(d["blk_kv_base"][b + 1])
            kvs = [InternalKV(k, t, v, int(d["kv_flags"][kv0 + j])) for j, (k, t, v) in enumerate(forward(d, b))]
            it = Iter(kvs, transforms=Transforms(seq, hide))
            scan, kv = [], it.First()
            while kv is not None:
                scan.append((kv.user_key, kv.trailer, kv.value))
                kv = it.Next()
            assert forward(x, b) == scan, (b, seq, hide)
