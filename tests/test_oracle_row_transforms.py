"""The row-format transforms of the oracle (orc_rowblk_decode_tf, the restatement
of rowblk.Iter under blockiter.Transforms) pinned the way the reference pins
its own: by iterating a block under a transform and the block physically
rewritten with the transform applied, and requiring the same KVs.

  TestBlockSyntheticPrefix (sstable/rowblk/rowblk_iter_test.go:288-356)
  TestBlockSyntheticSuffix (rowblk_iter_test.go:358-480)

restated for forward scans, plus the same differential form over raw keys:
rowblk.Iter puts the synthetic prefix into fullKey before the internal key is
decoded (rowblk_iter.go:259-263,400), so iterating raw keys r_i under prefix P
is iterating the raw keys P ++ r_i with no prefix.  That covers the cases the
reference's fixtures do not reach: a raw key shorter than 8 B made valid by
the prefix (its trailer then spans the prefix), Split of prefix ++ key (a
testkeys prefix holding '@' while the key has none; a cockroachkvs
version-length byte reaching into the prefix), hidden points and the value
prefix of keys whose kind comes from the prefix.
"""
import random

import pytest

import oracle
from pebble_amd.rowblk import Writer

PBL_SPLIT_WHOLE, PBL_SPLIT_TESTKEYS, PBL_SPLIT_CRDB = 0, 1, 2
FLAG_VALUE_PREFIX, FLAG_NO_VALUER = 0x1, 0x2


def scan(blk, flags=0, seq=0, hide=False, prefix=b"", suffix=b"", split=0):
    st, kvs, _ = oracle.rowblk_decode_block(blk, flags, (seq, hide, prefix, suffix, split))
    return st, [(k, t, v, f) for (k, t, v, f, _e) in kvs]


def ikey_block(keys, restarts):
    w = Writer(restarts)
    for k in keys:
        w.add(k.encode(), 0)  # base.InternalKey{UserKey: k} (rowblk_iter_test.go:482-484)
    return w.finish()


@pytest.mark.parametrize("prefix", ["_", "", "~", "fruits/"])
@pytest.mark.parametrize("restarts", [1, 2, 3, 4, 10])
def test_block_synthetic_prefix(prefix, restarts):
    keys = ["apple", "apricot", "banana", "grape", "orange", "peach", "pear", "persimmon"]
    elided = ikey_block(keys, restarts)
    included = ikey_block([prefix + k for k in keys], restarts)
    st_e, got = scan(elided, prefix=prefix.encode())
    st_i, exp = scan(included)
    assert st_e == st_i == 0
    assert got == exp and len(got) == len(keys)


@pytest.mark.parametrize("restarts", [1, 2, 3, 4, 10])
@pytest.mark.parametrize("replace_prefix", [False, True])
def test_block_synthetic_suffix(restarts, replace_prefix):
    keys = ["apple@2", "apricot@2", "banana@13", "cantaloupe", "grape@2", "orange@14", "peach@4", "pear@1",
            "persimmon@4"]
    pfx = "fruit/" if replace_prefix else ""
    got_blk = ikey_block(keys, restarts)
    exp_blk = ikey_block([pfx + k.split("@")[0] + "@15" for k in keys], restarts)
    st_g, got = scan(got_blk, prefix=pfx.encode(), suffix=b"@15", split=PBL_SPLIT_TESTKEYS)
    st_e, exp = scan(exp_blk)
    assert st_g == st_e == 0
    assert got == exp


def raw_block(raw_keys, values, restarts):
    w = Writer(restarts)
    for k, v in zip(raw_keys, values):
        w.add_raw(k, v)
    return w.finish()


def random_raw_keys(rng, n):
    """Raw internal keys of 1-20 bytes, a third shorter than 8; the first one
    at least 8 (readFirstKey, rowblk_iter.go:471-476).  Kind bytes are drawn
    from SET/DELETE/MERGE with the obsolete bit sometimes set; user-key bytes
    from a small alphabet holding '@' and small version-length bytes."""
    alpha = b"ab@\x00\x01\x02\x05\x09\x0d"
    keys = []
    for i in range(n):
        ln = rng.randint(8, 20) if i == 0 or rng.random() < 0.6 else rng.randint(1, 7)
        k = bytearray(rng.choice(alpha) for _ in range(ln))
        if ln >= 8 or rng.random() < 0.5:
            k[-8 if ln >= 8 else 0] = rng.choice([0, 1, 1, 2, 0x41, 0x40])  # a kind byte where it lands
        keys.append(bytes(k))
    return keys


def random_values(rng, n):
    return [bytes([rng.choice([0x00, 0x21, 0x80, 0xC0])]) + bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3])))
            if rng.random() < 0.9 else b"" for _ in range(n)]


PREFIXES = [b"\x01", b"pre@x", b"\x00\x00\x00\x00\x00\x00\x00\x01", b"ab\x09\x02", b"@", b"tenant-/\x05\x0d"]


@pytest.mark.parametrize("seed", range(12))
def test_raw_keys_under_prefix_equal_prefixed_raw_keys(seed):
    rng = random.Random(seed)
    for _ in range(6):
        n = rng.randint(1, 60)
        keys, vals = random_raw_keys(rng, n), random_values(rng, n)
        ri = rng.choice([1, 2, 3, 16])
        prefix = rng.choice(PREFIXES)
        suffix = rng.choice([b"", b"@9", b"\x00\x00\x00\x00\x00\x00\x00\x07\x09"])
        split = rng.choice([PBL_SPLIT_WHOLE, PBL_SPLIT_TESTKEYS, PBL_SPLIT_CRDB])
        seq = rng.choice([0, 77])
        hide = rng.random() < 0.5
        flags = rng.choice([0, FLAG_VALUE_PREFIX, FLAG_VALUE_PREFIX | FLAG_NO_VALUER])
        a = raw_block(keys, vals, ri)
        b = raw_block([prefix + k for k in keys], vals, ri)
        got = scan(a, flags, seq, hide, prefix, suffix, split)
        exp = scan(b, flags, seq, hide, b"", suffix, split)
        assert got == exp, (seed, prefix, suffix, split, seq, hide, flags)


def test_short_key_made_valid_by_prefix():
    """A 3-byte raw key under an 8-byte prefix: user key = prefix[:3], trailer =
    LE64(prefix[3:] ++ key) -- kind SET here, so the value prefix is stripped."""
    keys = [b"k" * 8 + (5 << 8 | 1).to_bytes(8, "little"), b"\x07\x08\x09"]
    vals = [b"\x00v0", b"\x00v1"]
    blk = raw_block(keys, vals, 16)
    prefix = b"PQR" + b"\x01\x00\x00\x00\x00"  # trailer bytes: 01 00 00 00 00 07 08 09
    st, kvs = scan(blk, FLAG_VALUE_PREFIX, prefix=prefix)
    assert st == 0
    assert kvs[1][0] == b"PQR"
    raw = int.from_bytes(b"\x01\x00\x00\x00\x00\x07\x08\x09", "little")
    assert kvs[1][1] == raw & ((((1 << 56) - 1) << 8) | 191)
    assert kvs[1][2] == b"v1" and not kvs[1][3] & 0x08
    # without the prefix the same entry is an invalid key with its whole value
    st, kvs = scan(blk, FLAG_VALUE_PREFIX)
    assert kvs[1] == (b"", 191, b"\x00v1", kvs[1][3]) and kvs[1][3] & 0x08


def test_split_sees_the_prefix():
    """testkeys: a prefix holding '@' and a key without one -> the suffix
    replaces everything from the prefix's '@' on.  cockroachkvs: a version
    length byte larger than the user key reaches into the prefix."""
    t = (0).to_bytes(8, "little")
    blk = raw_block([b"plain" + t, b"plaint" + t], [b"", b""], 16)
    st, kvs = scan(blk, prefix=b"a@b/", suffix=b"@5", split=PBL_SPLIT_TESTKEYS)
    assert st == 0 and [k for k, *_ in kvs] == [b"a@5", b"a@5"]
    blk = raw_block([b"ab\x05" + t], [b""], 16)
    st, kvs = scan(blk, prefix=b"xyzw", suffix=b"SFX", split=PBL_SPLIT_CRDB)
    assert st == 0 and kvs[0][0] == b"xy" + b"SFX"  # Split("xyzwab\x05") = 7 - 5 = 2


def test_seqnum_not_applied_to_invalid_keys():
    """SetSeqNum runs only on a decodable key (rowblk_iter.go:1168-1191)."""
    blk = raw_block([b"k" * 16, b"\x01"], [b"", b""], 16)
    st, kvs = scan(blk, seq=99)
    assert st == 0 and kvs[0][1] >> 8 == 99 and kvs[1][1] == 191
