"""Per-codec known-answer tests: the oracle's colblk column decoders
(oracle/colblk_oracle.c: dec_uints/u_at, dec_rawbytes, dec_bitmap,
dec_prefix + pb_parts) on every column the reference's own codec tests print,
against the values those tests wrote (tests/golden/make_colblk_fixtures.py):

  sstable/colblk/uints_test.go:71-257        testdata/uints        (widths 0/1/2/4/8, delta, offsets)
  sstable/colblk/raw_bytes_test.go:22        testdata/raw_bytes    (offsets 0-4, counts)
  sstable/colblk/prefix_bytes_test.go:27-224 testdata/prefix_bytes (bundles, duplicates, 2-byte offsets)
  sstable/colblk/bitmap_test.go:23-258       testdata/bitmap       (zero / default encodings, invert, rows)

The same bytes are decoded on the device in test_colblk_gpu.py
(test_codec_columns_in_device_blocks)."""
import json
import os

import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "colblk_golden.json")
with open(GOLDEN) as f:
    CODECS = json.load(f)["codecs"]

KIND = {"uints": oracle.COL_UINTS, "raw_bytes": oracle.COL_RAW_BYTES, "bitmap": oracle.COL_BITMAP,
        "prefix_bytes": oracle.COL_PREFIX_BYTES}


def cases():
    for codec, lst in CODECS.items():
        for e in lst:
            yield pytest.param(codec, e, id=f"{codec}:{e['source'].rsplit(':', 1)[1]}")


@pytest.mark.parametrize("codec,e", list(cases()))
def test_codec_kat(codec, e):
    buf = bytes.fromhex(e["bytes"])
    vals, end = oracle.col_decode(buf, e["offset"], e["rows"], KIND[codec])
    assert vals is not None, e["source"]
    exp = e["expect"]
    if codec in ("raw_bytes", "prefix_bytes"):
        exp = [bytes.fromhex(x) for x in exp]
    assert vals == exp, e["source"]
    # the decoder consumes exactly the column (a zero-row uints column is empty)
    assert end == len(buf), (e["source"], end, len(buf))


def test_every_codec_is_covered():
    assert {k: len(v) for k, v in CODECS.items()} == {"uints": 19, "raw_bytes": 11, "prefix_bytes": 12,
                                                       "bitmap": 25}
    # delta encodings, every width, non-zero offsets and 2-byte prefix-bytes offsets are among them
    dumps = "\n".join(e["dump"] for e in CODECS["uints"])
    for w in ("encoding: 1b", "encoding: 2b", "encoding: 4b", "encoding: 8b", "delta", "encoding: zero"):
        assert w in dumps, w
    assert any(e["offset"] for e in CODECS["raw_bytes"]) and any(e["offset"] for e in CODECS["bitmap"])
    assert any("encoding: 2b" in e["dump"] for e in CODECS["prefix_bytes"])


def embedded_blocks():
    """Every non-empty codec column embedded in a DefaultKeySchema data block
    (tests/colutil.py embed_column): uints as the trailers column, raw_bytes
    as the values column, bitmaps as isObsolete, prefix_bytes as the key-prefix
    column.  Returns [(codec, fixture, block)]."""
    from colutil import COL_OBSOLETE, COL_PREFIX, COL_TRAILERS, COL_VALUES, embed_column
    col = {"uints": COL_TRAILERS, "raw_bytes": COL_VALUES, "bitmap": COL_OBSOLETE, "prefix_bytes": COL_PREFIX}
    out = []
    for codec, lst in CODECS.items():
        for e in lst:
            if e["rows"] == 0:
                continue  # a data block has at least one row (an empty PrefixBytes panics)
            mk = max(len(bytes.fromhex(x)) for x in e["expect"]) if codec == "prefix_bytes" else 0
            blk = embed_column(col[codec], bytes.fromhex(e["bytes"])[e["offset"]:], e["offset"], e["rows"], mk)
            out.append((codec, e, blk))
    return out


def expected_field(codec, e):
    if codec in ("raw_bytes", "prefix_bytes"):
        return [bytes.fromhex(x) for x in e["expect"]]
    return list(e["expect"])


def decoded_field(codec, kvs):
    """kvs: (user_key, trailer, value, kv_flags, row) per row."""
    if codec == "uints":
        return [kv[1] for kv in kvs]
    if codec == "raw_bytes":
        return [kv[2] for kv in kvs]
    if codec == "bitmap":
        return [1 if kv[3] & 0x04 else 0 for kv in kvs]  # PBL_KV_OBSOLETE
    return [kv[0] for kv in kvs]


def test_codec_columns_in_blocks_oracle():
    blocks = embedded_blocks()
    assert len(blocks) == 67
    for codec, e, blk in blocks:
        st, kvs = oracle.colblk_decode_block(blk, 1)
        assert st == 0, e["source"]
        assert decoded_field(codec, kvs) == expected_field(codec, e), e["source"]
