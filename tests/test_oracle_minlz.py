"""The oracle's MinLZ restatement (oracle/minlz_oracle.c; compression indicator
8, internal/compression/minlz.go:52-72).

Pinned: the one property the reference's own test holds for this codec,
internal/compression/minlz_test.go:31-36 — a MinLZ decompressor decodes what
the Snappy fallback wrote (minlz.go:21-27).  The reference's Snappy-compressed
hamlet blocks (hamlet-sst/000002.sst), relabelled MinLZ, decode to exactly
h.txt's KVs.

PARITY UNPINNED: the MinLZ form itself.  No MinLZ-encoded bytes exist in
/root/reference (the codec, github.com/minio/minlz, is an absent dependency),
so the native-form tests below check the restatement against its own test
encoder (every op form, stored blocks, corrupt inputs), not against
minlz.Encode output."""
import random

import pytest

import oracle
from test_oracle_physical import PHYS, block_kvs, phys_bytes


def ops_of(block: bytes):
    """The op kinds of a MinLZ-form block (a walker independent of the C code)."""
    assert block[0] == 0
    i, n = 1, 0
    shift = 0
    while True:
        n |= (block[i] & 0x7F) << shift
        shift += 7
        i += 1
        if block[i - 1] < 0x80:
            break
    if n == 0:
        return {"stored"}
    kinds = set()
    while i < len(block):
        t = block[i]
        k = t & 3
        if k == 0:
            x = t >> 3
            nb = 0 if x < 29 else x - 28
            ln = x + 1 if x < 29 else 30 + int.from_bytes(block[i + 1:i + 1 + nb], "little")
            if t & 4:
                kinds.add("repeat")
                i += 1 + nb
            else:
                kinds.add("literal" if nb == 0 else f"literal+{nb}")
                i += 1 + nb + ln
        elif k == 1:
            ln = (t >> 2) & 15
            kinds.add("copy1" if ln < 15 else "copy1+1")
            i += 2 if ln < 15 else 3
        elif k == 2:
            ln = t >> 2
            nb = 0 if ln <= 60 else ln - 60
            kinds.add("copy2" if nb == 0 else f"copy2+{nb}")
            i += 3 + nb
        else:
            v = int.from_bytes(block[i:i + 4].ljust(4, b"\0"), "little")
            if t & 4:
                lits = (v >> 3) & 3
                ln = (v >> 5) & 63
                nb = 0 if ln <= 60 else ln - 60
                kinds.add("copy3" + (f"+{nb}" if nb else "") + ("+lits" if lits else ""))
                i += 4 + nb + lits
            else:
                kinds.add("copy2+lits")
                i += 3 + ((v >> 3) & 3) + 1
    return kinds


def corpus(rng, n):
    words = [rng.randbytes(rng.randrange(1, 12)) for _ in range(64)]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words) if rng.random() < 0.8 else rng.randbytes(rng.randrange(1, 70))
    return bytes(out[:n])


def test_snappy_fallback_blocks_decode_to_hamlet(golden):
    """minlz_test.go:31-36: the MinLZ decompressor decodes Snappy output."""
    blocks = []
    for b in PHYS["hamlet_snappy"]["blocks"]:
        raw = phys_bytes(b)[: b["length"]]
        assert raw[0] != 0
        assert oracle.minlz_decoded_len(raw) == b["decompressed_len"]
        d = oracle.minlz_decode(raw)
        assert d == oracle.snappy_decode(raw) and len(d) == b["decompressed_len"]
        blocks.append(d)
    assert block_kvs(blocks) == [tuple(x) for x in golden["hamlet_kvs"]]


@pytest.mark.parametrize("style", range(16))
def test_round_trips_every_style(style):
    rng = random.Random(style)
    srcs = [b"", b"a", b"abcd" * 100, rng.randbytes(5000), corpus(rng, 32768), bytes(rng.randrange(4) for _ in range(70000)),
            corpus(rng, 300_000), bytes(200) + rng.randbytes(100_000) + bytes(100_000)]
    for s in srcs:
        e = oracle.minlz_encode(s, style)
        assert e[0] == 0
        assert oracle.minlz_decoded_len(e) == len(s)
        assert oracle.minlz_decode(e) == s


def test_every_op_form_is_exercised():
    rng = random.Random(7)
    far = rng.randbytes(70_000)
    srcs = [corpus(rng, 40_000), bytes(rng.randrange(3) for _ in range(50_000)),
            far + rng.randbytes(50) + far[:5000] + rng.randbytes(3) + far[100:400],
            rng.randbytes(300) + bytes(70_000) + rng.randbytes(2000), b"xy" * 40_000 + rng.randbytes(90_000)]
    mid = rng.randbytes(3000)
    srcs += [mid * 3, mid + rng.randbytes(10) + mid[:200]]  # long copies at offsets past copy1's range
    seen = set()
    for style in (0, 1, 2, 3, 4, 6, 8):
        for s in srcs:
            e = oracle.minlz_encode(s, style)
            assert oracle.minlz_decode(e) == s
            seen |= ops_of(e)
    seen |= ops_of(oracle.minlz_encode(rng.randbytes(1000), 8))
    want = {"literal", "literal+1", "literal+2", "repeat", "copy1", "copy1+1", "copy2", "copy2+1", "copy2+2",
            "copy2+lits", "copy3", "copy3+lits", "stored"}
    assert want <= seen, want - seen


def test_corrupt_inputs_rejected():
    rng = random.Random(3)
    s = corpus(rng, 20_000)
    e = oracle.minlz_encode(s, 3)
    assert oracle.minlz_decode(b"") is None                        # no header
    assert oracle.minlz_decode(b"\x00") == b""                     # the empty block
    assert oracle.minlz_decode(e[: len(e) // 2]) is None           # truncated
    assert oracle.minlz_decode(b"\x00\x80") is None                # unterminated length
    assert oracle.minlz_decode(b"\x00\x00") is None                # stored, no bytes
    assert oracle.minlz_decode(b"\x00\x00abc") == b"abc"           # stored
    assert oracle.minlz_decode(b"\x00\x01\x08ab") is None          # output shorter than the block
    assert oracle.minlz_decode(b"\x00\x05\x05\x00") is None        # copy1 before any output
    assert oracle.minlz_decode(b"\x00\x05\x04") is None            # repeat (offset 1) before any output
    assert oracle.minlz_decode(b"\x00\x05\x00a\x04") is None       # repeat of 1 byte: output 2 != 5
    assert oracle.minlz_decode(b"\x00\x05\x00a\x1c") == b"aaaaa"   # repeat of 4 at offset 1
    assert oracle.minlz_decode(b"\x00" + bytes([0x81, 0x80, 0x80, 0x04])) is None  # > MaxBlockSize
    # one flipped byte anywhere decodes to other bytes or is rejected, never crashes
    for _ in range(300):
        b = bytearray(e)
        b[rng.randrange(1, len(b))] ^= 1 << rng.randrange(8)
        d = oracle.minlz_decode(bytes(b))
        assert d is None or isinstance(d, bytes)
