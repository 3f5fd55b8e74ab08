#!/usr/bin/env python3
"""Table-level fixtures, read as DATA from the reference
(run where /root/reference exists; the GPU box reads only the outputs):

  tests/golden/sst/*.sst   the reference's own test tables, copied byte for byte:
      hamlet-sst/000002.sst                     snappy, single-level index
      h-no-compression-sst/000012.sst           uncompressed, single-level
      h-no-compression-two-level-index-sst/000003.sst   two-level index
      h-zstd-compression-sst/000004.sst         zstd (not decoded on the device)
  tests/golden/sstable.json
      per table: the file size and the data-block handles (offset, length) found
      by an independent Python walk (footer -> index -> [lower index] -> handles,
      table.go:136-160,328-404); the KVs are h.txt's (sstable/test_fixtures.go)
      index_blocks: every `build` case of sstable/colblk/testdata/index_block:
      the block bytes rebuilt from the printed binfmt dump and the rows the test
      built it from (separator, offset, length, block properties)
"""
from __future__ import annotations

import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_colblk_fixtures import dump_to_bytes, parse_datadriven  # noqa: E402
from make_fixtures import REF, uvarint, walk_row_block_raw  # noqa: E402
from make_physical_fixtures import decompress  # noqa: E402

TABLES = {"hamlet_snappy": "sstable/testdata/hamlet-sst/000002.sst",
          "h_no_compression": "sstable/testdata/h-no-compression-sst/000012.sst",
          "h_two_level": "sstable/testdata/h-no-compression-two-level-index-sst/000003.sst",
          "h_zstd": "sstable/testdata/h-zstd-compression-sst/000004.sst"}


def block(data: bytes, h):
    o, ln = h
    return decompress(data[o + ln], data[o:o + ln])


def handles_of(blk: bytes):
    out = []
    for _k, v in walk_row_block_raw(blk):
        o, j = uvarint(v, 0)
        ln, _ = uvarint(v, j)
        out.append((o, ln))
    return out


def raw_kvs(blk: bytes) -> dict:
    return {k: v for k, v in walk_row_block_raw(blk)}


def table_case(path: str):
    data = open(path, "rb").read()
    footer = data[-53:]  # rocksDBFooterLen (these tables are Pebblev1-v4 / RocksDBv2)
    i = 1
    mo, i = uvarint(footer, i)
    ml, i = uvarint(footer, i)
    io_, i = uvarint(footer, i)
    il, i = uvarint(footer, i)
    meta = raw_kvs(block(data, (mo, ml)))
    po, j = uvarint(meta[b"rocksdb.properties"], 0)
    pl, _ = uvarint(meta[b"rocksdb.properties"], j)
    props = raw_kvs(block(data, (po, pl)))
    itype = uvarint(props.get(b"rocksdb.block.based.table.index.type", b"\0"), 0)[0]
    top = handles_of(block(data, (io_, il)))
    hs = top if itype != 2 else [h for t in top for h in handles_of(block(data, t))]
    return {"file": os.path.basename(path), "size": len(data), "checksum_type": footer[0],
            "metaindex": [mo, ml], "index": [io_, il], "index_type": itype,
            "version": int.from_bytes(data[-12:-8], "little"), "data_handles": hs}


def index_block_cases():
    out = []
    for c in parse_datadriven(os.path.join(REF, "sstable/colblk/testdata/index_block")):
        if not c["cmd"].startswith("build"):
            continue
        rows = []
        for line in c["input"].split("\n"):
            f = line.split()
            if len(f) >= 3:
                rows.append([f[0], int(f[1]), int(f[2]), f[3] if len(f) > 3 else ""])
        if "index-block-decoder" not in c["expected"]:
            continue
        dump = c["expected"][c["expected"].index("index-block-decoder"):]
        for a in c["cmd"].split()[1:]:  # `build rows=N`: Finish(N), the first N rows only
            if a.startswith("rows="):
                rows = rows[:int(a[5:])]
        out.append({"line": c["line"], "cmd": c["cmd"], "block_hex": dump_to_bytes(dump).hex(), "rows": rows})
    return out


def main():
    dst = os.path.join(HERE, "sst")
    os.makedirs(dst, exist_ok=True)
    res = {"tables": {}, "index_blocks": index_block_cases()}
    for name, rel in TABLES.items():
        src = os.path.join(REF, rel)
        shutil.copyfile(src, os.path.join(dst, f"{name}.sst"))
        try:
            res["tables"][name] = table_case(src) | {"file": f"{name}.sst", "source": rel}
        except ValueError:  # zstd blocks need a codec here too; record the file only
            data = open(src, "rb").read()
            res["tables"][name] = {"file": f"{name}.sst", "source": rel, "size": len(data)}
    with open(os.path.join(HERE, "sstable.json"), "w") as f:
        json.dump(res, f, indent=1)
    print({k: (v.get("index_type"), len(v.get("data_handles", []))) for k, v in res["tables"].items()},
          len(res["index_blocks"]), "index blocks")


if __name__ == "__main__":
    main()
