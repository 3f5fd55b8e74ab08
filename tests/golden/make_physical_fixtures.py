#!/usr/bin/env python3
"""Physical-block fixtures, read as DATA from the
reference's own test SSTs (run in the container that has /root/reference; the
GPU box only reads the generated physical.json / physical_blocks.bin):

  sstable/testdata/hamlet-sst/000002.sst              snappy-compressed data blocks
  sstable/testdata/h-zstd-compression-sst/000004.sst  zstd-compressed data blocks
  sstable/testdata/h-no-compression-sst/000012.sst    uncompressed data blocks
  sstable/testdata/h.txt                              their KVs (the independent oracle)

Every data block is kept as it sits in the file: the block bytes followed by
the 5-byte block trailer [compression indicator u8][checksum LE32]
(sstable/block/block.go:539-571, compression.go:170-193), with the file's
checksum type from its footer (block.go:106-114; all three are CRC32C).  The
walk to the data blocks (footer -> index block -> handles, table.go:189-404)
decompresses the INDEX blocks with pyarrow's snappy / zstd codecs: tooling
only, the data blocks are stored compressed, exactly as written by the
reference's writer.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_fixtures import REF, uvarint, walk_row_block_raw  # noqa: E402

FILES = [("hamlet_snappy", "sstable/testdata/hamlet-sst/000002.sst"),
         ("h_zstd", "sstable/testdata/h-zstd-compression-sst/000004.sst"),
         ("h_no_compression", "sstable/testdata/h-no-compression-sst/000012.sst")]


def decompress(indicator: int, b: bytes) -> bytes:
    import pyarrow as pa
    if indicator == 0:
        return b
    if indicator == 1:  # snappy: uvarint uncompressed length, then the elements
        n, _ = uvarint(b, 0)
        return pa.Codec("snappy").decompress(b, decompressed_size=n).to_pybytes()
    if indicator == 7:  # zstd frame (pebble prefixes the decoded length as a uvarint)
        n, i = uvarint(b, 0)
        return pa.Codec("zstd").decompress(b[i:], decompressed_size=n).to_pybytes()
    raise ValueError(indicator)


def physical_blocks(path: str):
    data = open(path, "rb").read()
    assert data[-8:] == b"\xf0\x9f\xaa\xb3\xf0\x9f\xaa\xb3"
    footer = data[-53:]
    checksum_type = footer[0]
    i = 1
    _mo, i = uvarint(footer, i)
    _ml, i = uvarint(footer, i)
    io_, i = uvarint(footer, i)
    il, i = uvarint(footer, i)
    index = decompress(data[io_ + il], data[io_:io_ + il])
    out = []
    for _k, v in walk_row_block_raw(index):
        o, j = uvarint(v, 0)
        ln, j = uvarint(v, j)
        phys = data[o:o + ln + 5]
        out.append({"offset_in_file": o, "length": ln, "indicator": phys[ln],
                    "checksum": int.from_bytes(phys[ln + 1:ln + 5], "little"), "bytes": phys,
                    "decompressed_len": len(decompress(phys[ln], phys[:ln]))})
    return checksum_type, out


def main():
    blob = bytearray()
    res = {}
    for name, rel in FILES:
        ct, blocks = physical_blocks(os.path.join(REF, rel))
        ent = []
        for bk in blocks:
            while len(blob) % 8:
                blob.append(0)
            ent.append({k: v for k, v in bk.items() if k != "bytes"} | {"blob_off": len(blob)})
            blob += bk["bytes"]
        res[name] = {"source": rel, "checksum_type": ct, "blocks": ent}
    with open(os.path.join(HERE, "physical_blocks.bin"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(HERE, "physical.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", {k: (v["checksum_type"], len(v["blocks"]), sorted({b["indicator"] for b in v["blocks"]}))
                    for k, v in res.items()}, len(blob), "bytes")


if __name__ == "__main__":
    main()
