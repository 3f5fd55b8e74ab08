"""Tables, CPU side: the oracle's footer and index-block
restatements pinned by the reference's own tables and index-block dumps
(tests/golden/make_sstable_fixtures.py), and the library's host-side
pbl_parse_footer (no GPU needed) against the oracle, including synthetic
Pebblev6/v7 footers with their footer checksum and corrupt footers."""
import ctypes
import json
import os
import random

import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "sstable.json")) as f:
    FIX = json.load(f)


def table_bytes(name):
    return open(os.path.join(GOLDEN, "sst", FIX["tables"][name]["file"]), "rb").read()


def lib_footer(buf, size):
    from pebble_amd import _native as N
    f = N.FooterC()
    rc = N.lib().pbl_parse_footer(bytes(buf), len(buf), size, ctypes.byref(f))
    if rc != 0:
        return rc, None
    return 0, {"table_format": f.table_format, "checksum_type": f.checksum_type, "attributes": f.attributes,
               "metaindex": (f.metaindex_off, f.metaindex_len), "index": (f.index_off, f.index_len),
               "footer": (f.footer_off, f.footer_len)}


@pytest.mark.parametrize("name", sorted(FIX["tables"]))
def test_footer_of_reference_tables(name):
    t = FIX["tables"][name]
    data = table_bytes(name)
    assert len(data) == t["size"]
    f = oracle.parse_footer(data[-61:], len(data))
    assert f["index"] == tuple(t["index"]) and f["checksum_type"] == t["checksum_type"]
    assert f["table_format"] == 2 + t["version"]
    rc, g = lib_footer(data[-61:], len(data))
    assert rc == 0 and g == f
    rc, g = lib_footer(data, len(data))  # the whole file as the buffer
    assert rc == 0 and g == f


def encode_footer(fmt, checksum, mh, ih, attributes=0):
    """footer.encode (sstable/table.go:406-460) for RocksDBv2 / Pebblev1-v8."""
    def uv(x):
        out = bytearray()
        while x >= 0x80:
            out.append((x & 0x7F) | 0x80)
            x >>= 7
        out.append(x)
        return bytes(out)
    flen = 61 if fmt >= 9 else 57 if fmt >= 8 else 53
    buf = bytearray(flen)
    buf[0] = checksum
    h = uv(mh[0]) + uv(mh[1]) + uv(ih[0]) + uv(ih[1])
    buf[1:1 + len(h)] = h
    magic = b"\xf7\xcf\xf4\x85\xb7\x41\xe2\x88" if fmt == 2 else b"\xf0\x9f\xaa\xb3\xf0\x9f\xaa\xb3"
    version = 2 if fmt == 2 else fmt - 2
    buf[-8:] = magic
    buf[-12:-8] = version.to_bytes(4, "little")
    if fmt >= 8:
        co = flen - 16
        if fmt >= 9:
            buf[co - 4:co] = attributes.to_bytes(4, "little")
        c = oracle.lib().orc_crc32c_update(0, bytes(buf[:co]), co)
        rest = bytes(buf[co + 4:])
        c = oracle.lib().orc_crc32c_update(c, rest, len(rest))
        v = ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF
        buf[co:co + 4] = v.to_bytes(4, "little")
    return bytes(buf)


@pytest.mark.parametrize("fmt", list(range(2, 11)))
def test_synthetic_footers_all_formats(fmt):
    rng = random.Random(fmt)
    size = 1 << 20
    for _ in range(20):
        mh = (rng.randrange(size // 2), rng.randrange(1, 5000))
        ih = (rng.randrange(size // 2), rng.choice([1, 127, 128, 300000 % (size // 2)]))
        ck = rng.choice([1, 3])
        buf = b"\xaa" * 13 + encode_footer(fmt, ck, mh, ih, rng.randrange(1 << 32))
        o = oracle.parse_footer(buf, size)
        assert o is not None and o["index"] == ih and o["metaindex"] == mh and o["table_format"] == fmt
        assert lib_footer(buf, size) == (0, o)
        # every single-byte corruption inside a checksummed footer is caught; in
        # any format the library and the oracle agree
        b = bytearray(buf)
        i = rng.randrange(13, len(b))
        b[i] ^= 1 << rng.randrange(8)
        o2 = oracle.parse_footer(bytes(b), size)
        rc, g = lib_footer(bytes(b), size)
        assert (o2 is None) == (rc == 12) and (o2 is None or g == o2)
        if fmt >= 8 and i < len(b) - 12:
            assert o2 is None


def test_corrupt_footers():
    data = table_bytes("h_no_compression")
    size = len(data)
    cases = [data[-61:-1] + b"\x00",               # bad magic
             data[-20:],                            # too short for a RocksDB footer
             data[-61:-12] + (9).to_bytes(4, "little") + data[-8:],   # unknown pebble version
             data[-53:][:0] + b"\x07" + data[-52:],  # unsupported checksum type
             ]
    for c in cases:
        assert oracle.parse_footer(c, size) is None
        assert lib_footer(c, size)[0] == 12
    # handles past the end of the file
    assert oracle.parse_footer(data[-61:], 27000) is None and lib_footer(data[-61:], 27000)[0] == 12


@pytest.mark.parametrize("name", ["hamlet_snappy", "h_no_compression", "h_two_level", "h_zstd"])
def test_row_index_walk_matches_fixture_handles(name):
    """Oracle index walk (row IndexIter + DecodeHandleWithProperties) down to the
    data blocks equals the fixture's independent walk."""
    import pyarrow as pa
    t = FIX["tables"][name]
    data = table_bytes(name)

    def block(h):
        o, ln = h
        raw, ind = data[o:o + ln], data[o + ln]
        if ind == 0:
            return raw
        n, i = oracle.go_uvarint(raw, 0)
        if ind == 1:
            return oracle.snappy_decode(raw)
        return pa.Codec("zstd").decompress(raw[i:], decompressed_size=n).to_pybytes()

    st, top = oracle.index_block_row(block(t["index"]))
    assert st == 0
    hs = [(o, ln) for o, ln, _p in top]
    if t["index_type"] == 2:
        lower = []
        for h in hs:
            st, e = oracle.index_block_row(block(h))
            assert st == 0
            lower += [(o, ln) for o, ln, _p in e]
        hs = lower
    assert hs == [tuple(x) for x in t["data_handles"]]


def test_colblk_index_block_dumps():
    for c in FIX["index_blocks"]:
        st, rows = oracle.index_block_col(bytes.fromhex(c["block_hex"]))
        assert st == 0
        assert rows == [(r[0].encode(), r[1], r[2], r[3].encode()) for r in c["rows"]], c["line"]
    # a column of the wrong type is a header corruption
    b = bytearray.fromhex(FIX["index_blocks"][0]["block_hex"])
    b[12] = 3  # col 1 (uint) claims bytes
    assert oracle.index_block_col(bytes(b))[0] == 4
