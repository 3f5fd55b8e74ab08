"""The native blockiter.Data adapter (pebble_amd/csrc/data_iter.cpp through
pebble_amd.blockiter.DataIter) on CPU: positioning over decoded arrays, checked
against the reference's rowblk_iter datadriven cases (TestBlockIter2,
rowblk_iter_test.go:123-161, sstable/rowblk/testdata/rowblk_iter), against the
host restatement pebble_amd.rowblk.Iter on random blocks, and the three
comparers against restatements of testkeys.compare (internal/testkeys/
testkeys.go:136-171) and cockroachkvs.Compare / Split (cockroachkvs.go:298-339).
The decoded arrays come from the oracle (test infrastructure); no GPU."""
import random
import struct

import numpy as np
import pytest

import oracle
from ddutil import parse_ikeys, run_iter_cmds
from pebble_amd import _native as N
from pebble_amd.blockiter import DataIter, key_compare, key_split
from pebble_amd.rowblk import InternalKV, Iter, Transforms, Writer, make_trailer


def decoded(blocks, flags=0):
    off, lens, pos = [], [], 0
    for b in blocks:
        off.append(pos)
        lens.append(len(b))
        pos += (len(b) + 15) // 16 * 16
    buf = np.zeros(pos + 16, np.uint8)
    for o, b in zip(off, blocks):
        buf[o:o + len(b)] = np.frombuffer(b, np.uint8)
    return oracle.rowblk_decode_batch(buf, np.array(off, np.uint64), np.array(lens, np.uint32), flags)


@pytest.mark.parametrize("ri", [1, 2, 3, 4])
def test_datadriven_rowblk_iter_cases(golden, ri):
    blk = None
    for case in golden["rowblk_iter_datadriven"]:
        cmd = case["cmd"].split()
        if cmd[0] == "build":
            w = Writer(ri)
            for k, s in parse_ikeys(case["input"]):
                w.add(k, make_trailer(s, 1), b"")
            blk = w.finish()
            continue
        gsn = 0
        for a in cmd[1:]:
            if a.startswith("globalSeqNum="):
                gsn = int(a.split("=")[1])
        d = decoded([blk])
        if gsn:  # (SyntheticSeqNum is applied by the decode: pbl_block_batch.synthetic_seq_num)
            d["trailer"] = (np.uint64(gsn) << np.uint64(8)) | (d["trailer"] & np.uint64(0xFF))
        it = DataIter(d, 0)
        assert it.status == 0
        assert run_iter_cmds(it, case["input"]) == case["expected"], case


def tk_compare(a: bytes, b: bytes) -> int:
    def split(k):
        i = k.rfind(b"@")
        return i if i >= 0 else len(k)

    ai, bi = split(a), split(b)
    if a[:ai] != b[:bi]:
        return -1 if a[:ai] < b[:bi] else 1
    sa, sb = a[ai:].removesuffix(b"_synthetic"), b[bi:].removesuffix(b"_synthetic")
    if not sa or not sb:
        return (len(sa) > len(sb)) - (len(sa) < len(sb))
    x, y = int(sa[1:]), int(sb[1:])
    return (y > x) - (y < x)


def crdb_compare(a: bytes, b: bytes) -> int:
    if not a or not b:
        return (len(a) > len(b)) - (len(a) < len(b))
    asl, bsl = a[-1], b[-1]
    pa, pb = a[:len(a) - asl], b[:len(b) - bsl]
    if pa != pb:
        return -1 if pa < pb else 1
    if asl == 0 or bsl == 0:
        return (asl > bsl) - (asl < bsl)

    def norm(s):
        v = s[:-1]
        if len(v) == 13:
            v = v[:12]
        if len(v) == 12 and v[8:] == b"\0\0\0\0":
            v = v[:8]
        return v

    x, y = norm(a[len(a) - asl:]), norm(b[len(b) - bsl:])
    return (y > x) - (y < x)  # descending versions: bytes.Compare(b, a)


def crdb_key(rng, roach):
    r = rng.random()
    if r < 0.2:
        return roach + b"\x00"  # no version
    if r < 0.6:
        return roach + b"\x00" + struct.pack(">Q", rng.choice([1, 5, 1 << 40, rng.getrandbits(63)])) + b"\x09"
    if r < 0.8:
        lg = rng.choice([0, 1, 7])
        return roach + b"\x00" + struct.pack(">QI", rng.choice([1, 5, 1 << 40]), lg) + b"\x0d"
    if r < 0.9:
        return roach + b"\x00" + struct.pack(">QI", rng.choice([1, 5]), 0) + b"\x01" + b"\x0e"
    return roach + b"\x00" + bytes(rng.getrandbits(8) for _ in range(17)) + b"\x12"  # lock-table version


def test_comparers_match_restatements():
    rng = random.Random(11)
    keys = [rng.choice([b"a", b"ab", b"b", b"a@", b""]) + (b"@" + str(rng.choice([0, 1, 5, 10, 99])).encode()
                                                            if rng.random() < 0.7 else b"")
            for _ in range(60)]
    keys = [k for k in keys if k.count(b"@") <= 1 and not k.endswith(b"@")]
    keys += [b"a@5_synthetic", b"a@5", b"b@10_synthetic"]
    for a in keys:
        for b in keys:
            assert key_compare(N.PBL_CMP_TESTKEYS, a, b) == tk_compare(a, b), (a, b)
            assert key_compare(N.PBL_CMP_DEFAULT, a, b) == (a > b) - (a < b)
    ck = [crdb_key(rng, rng.choice([b"k1", b"k2", b"k10", b"k"])) for _ in range(80)]
    for a in ck:
        assert key_split(N.PBL_CMP_CRDB, a) == len(a) - a[-1]
        for b in ck:
            assert key_compare(N.PBL_CMP_CRDB, a, b) == crdb_compare(a, b), (a.hex(), b.hex())
    assert key_split(N.PBL_CMP_TESTKEYS, b"abc@12") == 3 and key_split(N.PBL_CMP_TESTKEYS, b"abc") == 3
    assert key_split(N.PBL_CMP_DEFAULT, b"abc@12") == 6


def _random_block(rng, cmp, keyfn, n):
    import functools
    keys = sorted({keyfn() for _ in range(n)}, key=functools.cmp_to_key(cmp))
    w = Writer(rng.choice([1, 2, 4, 16]))
    kvs = []
    for k in keys:
        for s in sorted(rng.sample(range(1, 1000), rng.choice([1, 1, 2])), reverse=True):
            kind = rng.choice([1, 1, 0])
            obsolete = rng.random() < 0.2
            v = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 20])))
            w.add_with_optional_value_prefix(k, make_trailer(s, kind), obsolete, v, len(k), False, 0, False)
            kvs.append(k)
    return w.finish()


@pytest.mark.parametrize("comparer", [N.PBL_CMP_DEFAULT, N.PBL_CMP_TESTKEYS, N.PBL_CMP_CRDB])
def test_positioning_matches_host_iter(comparer):
    rng = random.Random(comparer + 3)
    cmp = {N.PBL_CMP_DEFAULT: lambda a, b: (a > b) - (a < b), N.PBL_CMP_TESTKEYS: tk_compare,
           N.PBL_CMP_CRDB: crdb_compare}[comparer]
    if comparer == N.PBL_CMP_TESTKEYS:
        keyfn = lambda: rng.choice([b"a", b"b", b"bb", b"c"]) + b"@" + str(rng.randrange(1, 30)).encode()  # noqa
    elif comparer == N.PBL_CMP_CRDB:
        keyfn = lambda: crdb_key(rng, rng.choice([b"k1", b"k2", b"k3"]))  # noqa: E731
    else:
        keyfn = lambda: bytes(rng.choice(b"abc") for _ in range(rng.randrange(1, 5)))  # noqa: E731
    blocks = [_random_block(rng, cmp, keyfn, rng.randrange(1, 60)) for _ in range(6)] + [Writer(16).finish()]
    d = decoded(blocks)
    for b in range(len(blocks)):
        st, kvs, _ = oracle.rowblk_decode_block(blocks[b])
        for hide in (False, True):
            ref = Iter([InternalKV(k, t, v, f) for k, t, v, f, _o in kvs], cmp=cmp,
                       transforms=Transforms(hide_obsolete_points=hide))
            it = DataIter(d, b, comparer, hide)
            assert it.status == 0
            probes = [kv[0] for kv in kvs] + [keyfn() for _ in range(10)] + [b""]
            ops = []
            for _ in range(300):
                r = rng.random()
                if r < 0.25:
                    ops.append(("SeekGE", rng.choice(probes)))
                elif r < 0.4:
                    ops.append(("SeekLT", rng.choice(probes)))
                else:
                    ops.append((rng.choice(["Next", "Prev", "First", "Last"]), None))
            for op, arg in ops:
                a = getattr(it, op)(arg) if arg is not None else getattr(it, op)()
                e = getattr(ref, op)(arg) if arg is not None else getattr(ref, op)()
                assert a == e, (b, op, arg, a, e)
                assert it.Valid() == ref.Valid()


def test_prefix_ops_and_invalidate():
    keys = [b"a@3", b"a@2", b"a@1", b"b@9", b"b@1", b"c@4"]
    w = Writer(2)
    for i, k in enumerate(keys):
        w.add(k, make_trailer(10 - i, 1), b"v%d" % i)
    d = decoded([w.finish()])
    it = DataIter(d, 0, N.PBL_CMP_TESTKEYS)
    # SeekPrefixGE (rowblk_iter.go:550-564)
    kv, miss = it.SeekPrefixGE(b"a@2")
    assert kv.user_key == b"a@2" and not miss
    kv, miss = it.SeekPrefixGE(b"a@0")  # lands on b@9: positioned, prefix differs
    assert kv is None and miss and it.KV().user_key == b"b@9"
    kv, miss = it.SeekPrefixGE(b"d@1")
    assert kv is None and not miss
    # NextWithSamePrefix (:571-598): stays on the new-prefix key when exhausted
    it.First()
    assert [it.NextWithSamePrefix()[0].user_key for _ in range(2)] == [b"a@2", b"a@1"]
    kv, ex = it.NextWithSamePrefix()
    assert kv is None and ex and it.KV().user_key == b"b@9"
    kv, ex = it.NextWithSamePrefix()
    assert kv.user_key == b"b@1" and not ex
    # NextPrefix (:1204-1218): the first key >= succKey after the current one
    it.First()
    assert it.NextPrefix(b"b").user_key == b"b@9"
    assert it.NextPrefix(b"c").user_key == b"c@4"
    assert it.NextPrefix(b"d") is None
    # IsLowerBound (:542-545)
    assert it.IsLowerBound(b"a@5") and it.IsLowerBound(b"a") and not it.IsLowerBound(b"a@1")
    # Invalidate / IsDataInvalidated (block_iter.go:96-105)
    assert not it.IsDataInvalidated()
    it.Invalidate()
    assert it.IsDataInvalidated() and it.First() is None and not it.Valid()


def test_corrupt_block_reports_its_status():
    d = decoded([b"\x00\x00\x00\x00", Writer(16).finish()])
    assert DataIter(d, 0).status == int(d["blk_status"][0]) != 0
    assert DataIter(d, 1).status == 0 and DataIter(d, 1).First() is None
