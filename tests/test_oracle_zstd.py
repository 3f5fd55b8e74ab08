"""The oracle's zstd restatement (oracle/zstd_oracle.c, RFC 8878 as decoded by
DataDog/zstd v1.5.7 = facebook/zstd 1.5.7, the library Pebble's
zstdDecompressor calls: internal/compression/zstd_cgo.go:86-108), pinned by

  * the reference's zstd table, sstable/testdata/h-zstd-compression-sst/000004.sst:
    every data block decodes to blocks whose KVs are exactly h.txt's;
  * frames written by facebook/zstd itself (the codec pyarrow bundles) at
    levels -5..19 over random, repetitive and text-like inputs, exercising
    raw / RLE / compressed blocks, raw / RLE / Huffman / treeless literals with
    1 and 4 streams, and predefined / RLE / FSE / repeat sequence tables;
  * XXH64 against the xxhash package (the content checksum);
and corrupt inputs (truncations, flipped bytes) never decode to a wrong length."""
import json
import os
import random

import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "physical.json")) as f:
    PHYS = json.load(f)
BLOB = open(os.path.join(GOLDEN, "physical_blocks.bin"), "rb").read()


def zstd(data: bytes, level: int, checksum: bool = False) -> bytes:
    import pyarrow as pa
    return pa.Codec("zstd", compression_level=level).compress(data, asbytes=True)


def corpus(rng, kind, n):
    words = [bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(2, 9))) for _ in range(300)]
    if kind == 0:
        return rng.randbytes(n)
    if kind == 1:
        return b" ".join(rng.choice(words) for _ in range(n // 5 + 1))[:n]
    if kind == 2:
        return bytes([rng.choice(b"ab")]) * n
    return b"".join(rng.choice(words) + rng.randbytes(rng.randint(0, 3)) for _ in range(n // 6 + 1))[:n]


def test_h_zstd_blocks_decode_to_hamlet(golden):
    blocks = []
    for b in PHYS["h_zstd"]["blocks"]:
        assert b["indicator"] == 7
        raw = BLOB[b["blob_off"]: b["blob_off"] + b["length"]]
        d = oracle.zstd_block(raw)
        assert not isinstance(d, int) and len(d) == b["decompressed_len"]
        blocks.append(d)
    kvs = []
    for blk in blocks:
        st, kv, _ = oracle.rowblk_decode_block(blk)
        assert st == 0
        kvs += [(k.decode(), v.decode()) for k, _t, v, _f, _e in kv]
    assert kvs == [tuple(x) for x in golden["hamlet_kvs"]]


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
def test_frames_from_the_zstd_library(level):
    rng = random.Random(level + 100)
    for trial in range(60):
        n = rng.choice([0, 1, 5, 100, 1000, 5000, 32768, 70000, 140000])
        data = corpus(rng, trial % 4, n)
        c = zstd(data, level)
        assert oracle.zstd_decompress(c, len(data) + 8) == data, (trial, n)
        if n:
            assert oracle.zstd_decompress(c, len(data) - 1) == -3  # output too small


def test_xxh64_against_xxhash():
    import xxhash
    rng = random.Random(2)
    for n in [0, 1, 3, 4, 7, 8, 31, 32, 33, 63, 64, 100, 1000, 4097]:
        d = rng.randbytes(n)
        for seed in (0, 1, 2**63 + 5):
            assert oracle.lib().orc_xxh64(d, len(d), seed) == xxhash.xxh64(d, seed=seed).intdigest()


def test_frame_header_forms():
    """Skippable frames are passed over, frames concatenate, a dictionary ID is
    unsupported, the reserved bit and a bad magic are corrupt."""
    a, b = b"hello hello hello", b"world" * 50
    fa, fb = zstd(a, 3), zstd(b, 3)
    skip = (0x184D2A53).to_bytes(4, "little") + (3).to_bytes(4, "little") + b"xyz"
    assert oracle.zstd_decompress(skip + fa + fb, 1000) == a + b
    bad = bytearray(fa)
    bad[4] |= 8
    assert oracle.zstd_decompress(bytes(bad), 1000) == -1
    assert oracle.zstd_decompress(b"\x00" + fa[1:], 1000) == -1
    d = bytearray(fa)
    d[4] = (d[4] & ~3) | 1  # a 1-byte dictionary ID follows
    d.insert(5 + (0 if d[4] & 0x20 else 1), 7)
    assert oracle.zstd_decompress(bytes(d), 1000) == -2


def test_corrupt_frames_never_decode_wrong():
    rng = random.Random(4)
    for trial in range(300):
        data = corpus(rng, 1 + trial % 3, rng.randrange(1, 20000))
        c = bytearray(zstd(data, rng.choice([1, 3, 9])))
        m = trial % 3
        if m == 0:
            c = c[: rng.randrange(1, len(c))]
        elif m == 1:
            c[rng.randrange(4, len(c))] ^= 1 << rng.randrange(8)
        else:
            c = c + bytes(rng.randrange(1, 4))
        out = oracle.zstd_decompress(bytes(c), len(data))
        # a flipped bit inside a literal or a raw block can decode to other bytes
        # of the same length; anything that is not an error has the frame's size
        assert isinstance(out, int) or len(out) == len(data), trial
