"""The oracle's fused HideObsoletePoints decode (decode_batch with
PBL_ROW_HIDE_OBSOLETE: rowblk.Iter under blockiter.Transforms
{HideObsoletePoints}, rowblk_iter.go:1168-1179) against the transform
restatement over the plain decode (oracle.transform_batch, pinned by the
reference's transform scans): the same KVs for every block both decode."""
import random

import numpy as np

import oracle
from pebble_amd import _native as N
from rowutil import mvcc_block
from test_rowblk_gpu import pack, random_block

HIDE = N.PBL_ROW_HIDE_OBSOLETE
KEYS = ("trailer", "kv_flags", "entry_off", "key_off", "val_off", "key_bytes", "val_bytes")


def per_block(r, b):
    kv0, kv1 = int(r["blk_kv_base"][b]), int(r["blk_kv_base"][b + 1])
    ko = r["key_off"][kv0 + b: kv1 + b + 1]
    vo = r["val_off"][kv0 + b: kv1 + b + 1]
    kb, vb = int(r["blk_key_base"][b]), int(r["blk_val_base"][b])
    return [(bytes(r["key_bytes"][kb + ko[j]: kb + ko[j + 1]]), int(r["trailer"][kv0 + j]),
             bytes(r["val_bytes"][vb + vo[j]: vb + vo[j + 1]]), int(r["kv_flags"][kv0 + j]),
             int(r["entry_off"][kv0 + j])) for j in range(kv1 - kv0)]


def test_fused_hide_matches_transform_restatement():
    rng = random.Random(5)
    blocks = [random_block(rng)[0] for _ in range(150)] + [mvcc_block(rng, rng.randint(1, 300), rng.choice([1, 4, 16]),
                                                                     rng.random() < 0.5, rng.random() < 0.7)
                                                          for _ in range(100)]
    for flags in (0, N.PBL_ROW_VALUE_PREFIX, N.PBL_ROW_VALUE_PREFIX | N.PBL_ROW_NO_VALUER):
        buf, off, lens = pack(blocks)
        plain = oracle.decode_batch(buf, off, lens, 0, None, flags)
        fused = oracle.decode_batch(buf, off, lens, 0, None, flags | HIDE)
        tf = oracle.transform_batch(plain, 0, True, src=(buf, off, lens, 0, None, flags))
        n_hidden = 0
        for b in range(len(blocks)):
            if plain["blk_status"][b] == 0:
                assert fused["blk_status"][b] == 0
                assert per_block(fused, b) == per_block(tf, b), (flags, b)
                n_hidden += int(plain["blk_kv_base"][b + 1] - plain["blk_kv_base"][b]) - \
                    int(fused["blk_kv_base"][b + 1] - fused["blk_kv_base"][b])
        assert n_hidden > 100
        # restart words are kept; raw keys ignore the flag
        assert np.array_equal(oracle.decode_batch(buf, off, lens, 0, None, N.PBL_ROW_RAW_KEYS | HIDE)["key_bytes"],
                              oracle.decode_batch(buf, off, lens, 0, None, N.PBL_ROW_RAW_KEYS)["key_bytes"])


def test_hidden_point_with_empty_set_value_iterates():
    """Go skips a hidden point before reading its value (rowblk_iter.go:1168-1199):
    an empty SET value on an obsolete point fails the plain decode under value
    prefixes, not the hiding one."""
    from pebble_amd.rowblk import Writer, make_trailer
    w = Writer(16)
    w.add_with_optional_value_prefix(b"a", make_trailer(5, 1), False, b"x", 1, True, 0, False)
    w.add_with_optional_value_prefix(b"b", make_trailer(4, 1), True, b"", 1, False, 0, False)
    w.add_with_optional_value_prefix(b"c", make_trailer(3, 1), False, b"y", 1, True, 0, False)
    buf, off, lens = pack([w.finish()])
    assert oracle.decode_batch(buf, off, lens, 0, None, N.PBL_ROW_VALUE_PREFIX)["blk_status"][0] != 0
    r = oracle.decode_batch(buf, off, lens, 0, None, N.PBL_ROW_VALUE_PREFIX | HIDE)
    assert r["blk_status"][0] == 0 and r["n_kv"] == 2


def test_fused_hide_colblk_and_mixed_match_transform_restatement():
    """Colblk blocks under the flag (DataBlockIter, data_block.go:1680-1697:
    isObsolete rows skipped) and mixed row + colblk batches: the oracle's fused
    decode equals the transform restatement over its plain decode, array for
    array (the mixed GPU test checks the device against the fused form)."""
    from colutil import build_block, random_rows
    from pebble_amd.colblk import SCHEMA_CRDB1, SCHEMA_DEFAULT
    rng = random.Random(7)
    blocks, fmts = [], []
    for i in range(120):
        if i % 3 == 2:
            blocks.append(mvcc_block(rng, rng.randint(1, 200), rng.choice([1, 4, 16]), rng.random() < 0.5,
                                     rng.random() < 0.7))
            fmts.append(N.PBL_FMT_ROW)
        else:
            schema = SCHEMA_DEFAULT if i % 3 == 0 else SCHEMA_CRDB1
            rows = random_rows(rng, schema, rng.choice([1, 5, 17, 100, 300]), shared=rng.choice([0, 3]),
                               val_len=(0, rng.choice([3, 50, 400])))
            blocks.append(build_block(schema, rows, rng.choice([1, 4, 16]))[0])
            fmts.append(schema)
    for i in range(0, 120, 29):  # a few corrupt blocks stay failed
        b = bytearray(blocks[i])
        b[rng.randrange(len(b))] ^= 0x5A
        blocks[i] = bytes(b)
    buf, off, lens = pack(blocks)
    bf = np.array(fmts, np.uint8)
    for flags in (0, N.PBL_ROW_VALUE_PREFIX):
        plain = oracle.decode_batch(buf, off, lens, 0, bf, flags)
        fused = oracle.decode_batch(buf, off, lens, 0, bf, flags | HIDE)
        tf = oracle.transform_batch(plain, 0, True, src=(buf, off, lens, 0, bf, flags))
        assert list(fused["blk_status"]) == list(tf["blk_status"])
        hidden = 0
        for b in range(len(blocks)):
            if fused["blk_status"][b] == 0:
                assert per_block(fused, b) == per_block(tf, b), (flags, b)
                hidden += len(per_block(plain, b)) - len(per_block(fused, b))
        assert hidden > 0
    # a colblk-only batch as well (the single-format colblk path's contract)
    cb = [blk for blk, f in zip(blocks, fmts) if f == SCHEMA_CRDB1]
    buf, off, lens = pack(cb)
    plain = oracle.decode_batch(buf, off, lens, SCHEMA_CRDB1, None, 0)
    fused = oracle.decode_batch(buf, off, lens, SCHEMA_CRDB1, None, HIDE)
    tf = oracle.transform_batch(plain, 0, True)
    for k in KEYS + ("blk_kv_base", "blk_key_base", "blk_val_base", "blk_status"):
        assert np.array_equal(fused[k], tf[k]), k
