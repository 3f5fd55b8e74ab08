#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the
reference's own test data (run once in the container that has /root/reference;
the GPU box only reads the generated files).

Sources (cockroachdb/pebble, read as data):
  sstable/rowblk/rowblk_writer_test.go:51-55, 104-114  exact row-block bytes
  sstable/rowblk/unsafe_test.go:21-33                  varint known answers
  sstable/rowblk/testdata/rowblk_iter                  datadriven iterator cases
  sstable/testdata/h-no-compression-sst/000012.sst     real row-format SST (Pebblev1, 2 KiB blocks)
  sstable/testdata/h-no-compression-two-level-index-sst/000003.sst
  sstable/testdata/h.txt                               word counts: the independent oracle for the SSTs
                                                       (sstable/test_fixtures.go:46-76: key = s[8:], value = s[:8])
  colblk / cockroachkvs datadriven hex dumps           see make_colblk_fixtures() below

The SST walk here only locates data blocks (footer -> index block -> block
handles, sstable/table.go:189-404, sstable/block/block.go:80-87); it never
decodes data blocks, so the fixtures stay independent of the oracle.
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def uvarint(b: bytes, i: int):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        if c < 0x80:
            return x, i
        s += 7


def walk_row_block_raw(blk: bytes):
    """Minimal RawIter-style walk used ONLY for index blocks (keys -> handles)."""
    nres = int.from_bytes(blk[-4:], "little")
    end = len(blk) - 4 * (1 + nres)
    off, key = 0, b""
    while off < end:
        sh, off = uvarint(blk, off)
        un, off = uvarint(blk, off)
        vl, off = uvarint(blk, off)
        key = key[:sh] + blk[off:off + un]
        off += un
        yield key, blk[off:off + vl]
        off += vl


def sst_data_blocks(path: str):
    data = open(path, "rb").read()
    magic = data[-8:]
    assert magic in (b"\xf7\xcf\xf4\x85\xb7\x41\xe2\x88", b"\xf0\x9f\xaa\xb3\xf0\x9f\xaa\xb3"), magic
    footer = data[-53:]  # rocksDBFooterLen = 1 + 2*20 + 4 + 8 (Pebblev1..v5)
    i = 1
    _mo, i = uvarint(footer, i)
    _ml, i = uvarint(footer, i)
    io_, i = uvarint(footer, i)
    il, i = uvarint(footer, i)
    index = data[io_:io_ + il]
    handles = []
    for _k, v in walk_row_block_raw(index):
        o, j = uvarint(v, 0)
        ln, j = uvarint(v, j)
        handles.append((o, ln))
    # two-level index: top-level entries point at index blocks, not data blocks
    second = []
    for o, ln in handles:
        blk = data[o:o + ln]
        # heuristic-free check: an index block's values are varint handles that
        # point back into the file before the index
        try:
            inner = [(uvarint(v, 0), v) for _k, v in walk_row_block_raw(blk)]
            ok = all(len(v) >= 2 for _x, v in inner) and path.endswith("000003.sst")
        except Exception:
            ok = False
        if ok:
            for _k, v in walk_row_block_raw(blk):
                o2, j = uvarint(v, 0)
                l2, j = uvarint(v, j)
                second.append((o2, l2))
    if second:
        handles = second
    blocks = []
    for o, ln in handles:
        assert data[o + ln] == 0, "fixture SSTs are uncompressed"  # block type byte
        blocks.append(data[o:o + ln])
    return blocks


def hamlet_expected():
    kv = {}
    with open(os.path.join(REF, "sstable/testdata/h.txt"), "rb") as f:
        for line in f:
            kv[line[8:].strip()] = line[:8].strip()
    assert len(kv) == 1710
    return [[k.decode(), kv[k].decode()] for k in sorted(kv)]


def parse_datadriven(path: str):
    """cockroachdb/datadriven file format: `cmd args\\ninput\\n----\\nexpected\\n\\n`."""
    cases, lines, i = [], open(path).read().split("\n"), 0
    while i < len(lines):
        if not lines[i].strip() or lines[i].startswith("#"):
            i += 1
            continue
        cmd = lines[i]
        i += 1
        inp = []
        while i < len(lines) and lines[i] != "----":
            inp.append(lines[i])
            i += 1
        i += 1
        out = []
        if i < len(lines) and lines[i] == "----":  # double-separator form
            i += 1
            while i < len(lines) and not (lines[i] == "----" and i + 1 < len(lines) and lines[i + 1] == "----"):
                out.append(lines[i])
                i += 1
            i += 2
        else:
            while i < len(lines) and lines[i].strip() != "":
                out.append(lines[i])
                i += 1
        cases.append({"cmd": cmd, "input": "\n".join(inp), "expected": "\n".join(out)})
    return cases


def main():
    out = {}
    # exact bytes (rowblk_writer_test.go:51-55 and :104-114)
    out["writer_basic"] = {
        "restart_interval": 16,
        "raw_kvs": [["apple", ""], ["apricot", ""], ["banana", ""]],
        "block_hex": (b"\x00\x05\x00apple" b"\x02\x05\x00ricot" b"\x00\x06\x00banana"
                      b"\x00\x00\x00\x00\x01\x00\x00\x00").hex(),
    }
    out["writer_with_prefix"] = {
        "restart_interval": 2,
        # (user key, value, addValuePrefix, valuePrefix, setHasSameKeyPrefix); ikey() in the
        # test (rowblk_iter_test.go:482) is the zero trailer.
        "adds": [["apple", "red", False, 0, True], ["apricot", "orange", True, 0xFF, False],
                 ["banana", "yellow", True, 0x00, True], ["cherry", "red", False, 0, True],
                 ["mango", "juicy", False, 0, True]],
        "block_hex": (b"\x00\x0d\x03apple\x00\x00\x00\x00\x00\x00\x00\x00red"
                      b"\x02\x0d\x07ricot\x00\x00\x00\x00\x00\x00\x00\x00\xfforange"
                      b"\x00\x0e\x07banana\x00\x00\x00\x00\x00\x00\x00\x00\x00yellow"
                      b"\x00\x0e\x03cherry\x00\x00\x00\x00\x00\x00\x00\x00red"
                      b"\x00\x0d\x05mango\x00\x00\x00\x00\x00\x00\x00\x00juicy"
                      b"\x00\x00\x00\x00\x2a\x00\x00\x00\x56\x00\x00\x80\x03\x00\x00\x00").hex(),
    }
    out["varint_kat"] = [0, 1, 1 << 7, 1 << 8, 1 << 14, 1 << 15, 1 << 20, 1 << 21, 1 << 28, 1 << 29, 1 << 31]
    out["rowblk_iter_datadriven"] = parse_datadriven(os.path.join(REF, "sstable/rowblk/testdata/rowblk_iter"))

    # real SSTs
    for name, rel in [("h_no_compression", "sstable/testdata/h-no-compression-sst/000012.sst")]:
        blocks = sst_data_blocks(os.path.join(REF, rel))
        blob = bytearray()
        offs, lens = [], []
        for bk in blocks:
            while len(blob) % 8:
                blob.append(0)
            offs.append(len(blob))
            lens.append(len(bk))
            blob += bk
        with open(os.path.join(HERE, f"{name}_blocks.bin"), "wb") as f:
            f.write(bytes(blob))
        out[name] = {"source": rel, "block_off": offs, "block_len": lens}
    out["hamlet_kvs"] = hamlet_expected()

    with open(os.path.join(HERE, "rowblk_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "rowblk_golden.json"))
    if "--colblk" in sys.argv or True:
        try:
            from make_colblk_fixtures import main as colmain  # type: ignore
        except ImportError:
            return
        colmain()


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    main()
