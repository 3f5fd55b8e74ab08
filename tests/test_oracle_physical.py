"""The oracle's physical-block step (oracle/physical_oracle.c) pinned by the
reference's own SSTs (tests/golden/make_physical_fixtures.py): every data
block's stored CRC32C checksum (sstable/block/block.go:164-197,
internal/crc/crc.go), snappy decompression of hamlet-sst/000002.sst to blocks
whose KVs are exactly h.txt's (sstable/test_fixtures.go:46-76), and the XXH64
checksum form against the published XXH64 vectors."""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "physical.json")) as f:
    PHYS = json.load(f)
BLOB = open(os.path.join(GOLDEN, "physical_blocks.bin"), "rb").read()


def phys_bytes(b):
    return BLOB[b["blob_off"]: b["blob_off"] + b["length"] + 5]


def block_kvs(blocks):
    """(user key, value) of row blocks, via the oracle's row decoder."""
    kvs = []
    for blk in blocks:
        st, kv, _ = oracle.rowblk_decode_block(blk)
        assert st == 0
        kvs += [(k.decode(), v.decode()) for k, _t, v, _f, _e in kv]
    return kvs


@pytest.mark.parametrize("name", sorted(PHYS))
def test_crc32c_matches_stored_checksums(name):
    f = PHYS[name]
    assert f["checksum_type"] == 1  # CRC32C
    for b in f["blocks"]:
        p = phys_bytes(b)
        assert oracle.block_checksum(1, p[: b["length"] + 1]) == b["checksum"]
        bad = bytearray(p)
        bad[len(bad) // 3] ^= 0x10
        assert oracle.block_checksum(1, bytes(bad[: b["length"] + 1])) != b["checksum"]


def test_snappy_blocks_decode_to_hamlet(golden):
    f = PHYS["hamlet_snappy"]
    blocks = []
    for b in f["blocks"]:
        assert b["indicator"] == 1
        d = oracle.snappy_decode(phys_bytes(b)[: b["length"]])
        assert d is not None and len(d) == b["decompressed_len"]
        blocks.append(d)
    assert block_kvs(blocks) == [tuple(x) for x in golden["hamlet_kvs"]]


def test_uncompressed_and_zstd_files_hold_the_same_kvs(golden):
    """The zstd file is decompressed with pyarrow's zstd (tooling: zstd is not
    decoded on the device); both files hold h.txt's KVs."""
    import pyarrow as pa
    for name, dec in (("h_no_compression", lambda b: b),
                      ("h_zstd", None)):
        blocks = []
        for b in PHYS[name]["blocks"]:
            raw = phys_bytes(b)[: b["length"]]
            if dec is None:
                n, i = 0, 0
                shift = 0
                while True:
                    n |= (raw[i] & 0x7F) << shift
                    shift += 7
                    i += 1
                    if raw[i - 1] < 0x80:
                        break
                blocks.append(pa.Codec("zstd").decompress(raw[i:], decompressed_size=n).to_pybytes())
            else:
                blocks.append(raw)
        assert block_kvs(blocks) == [tuple(x) for x in golden["hamlet_kvs"]]


def test_snappy_corrupt_inputs_rejected():
    b = PHYS["hamlet_snappy"]["blocks"][0]
    raw = phys_bytes(b)[: b["length"]]
    assert oracle.snappy_decode(raw[: len(raw) // 2]) is None      # truncated
    assert oracle.snappy_decode(b"\x05\x01\x00") is None           # copy before any output
    assert oracle.snappy_decode(b"\x03" + b"\x08abc") == b"abc"    # 3-byte literal
    assert oracle.snappy_decode(b"\x08\x00a\x0d\x01") == b"aaaaaaaa"  # overlapping copy (offset 1)


def test_xxh64_vectors():
    # XXH64 reference vectors (seed 0): "", "a", "abc"
    import xxhash
    for s, h in ((b"", 0xEF46DB3751D8E999), (b"a", 0xD24EC4F1A98C6E5B), (b"abc", 0x44BC2CF5AD770999)):
        assert xxhash.xxh64(s).intdigest() == h
        assert oracle.xxhash64_checksum(s) == h & 0xFFFFFFFF
