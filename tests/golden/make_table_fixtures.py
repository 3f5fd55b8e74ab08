#!/usr/bin/env python3
"""Columnar (Pebblev7) tables and their expected scans, read from the reference
AS DATA (test infrastructure; run once in the build container, outputs
committed):

  tool/testdata/cr-schema-sst/000014.sst            -> tests/golden/sst/cr_schema_000014.sst
  tool/testdata/find-val-sep-db/0000{05,08,11}.sst  -> tests/golden/sst/find_val_sep_0000NN.sst
  tool/testdata/sstable_scan (the `sstable scan` outputs of those files)
                                                    -> tests/golden/tables.json

The scan lines print keys with each table's comparer: CockroachDB keys as
roachkey[@wall.nanos,logical] (cockroachkvs.FormatKey, cockroachkvs.go:1111-1160),
re-encoded here with EncodeTimestamp (:174-197); other keys Go-quoted.  Values
print as hex, blob handles as (fREF,blkB,idI,lenL) (sstable/blob/handle.go:98-100).
"""
import json
import os
import re
import struct

REF = "/root/reference/tool/testdata/sstable_scan"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables.json")
KINDS = {"SET": 1, "DEL": 0, "MERGE": 2, "SINGLEDEL": 7, "SETWITHDEL": 18, "DELSIZED": 23}


def crdb_key(s: str) -> bytes:
    """cockroachkvs.EncodeTimestamp of a FormatKey string."""
    if "@" not in s:
        return s.encode() + b"\x00"
    roach, ver = s.split("@", 1)
    wall_s, logical = ver.split(",")
    if "." in wall_s:
        sec, ns = wall_s.split(".")
        wall = int(sec) * 10**9 + int(ns)
    else:
        wall = int(wall_s) * 10**9
    logical = int(logical)
    if logical == 0:
        if wall == 0:
            return roach.encode() + b"\x00"
        return roach.encode() + b"\x00" + struct.pack(">Q", wall) + b"\x09"
    return roach.encode() + b"\x00" + struct.pack(">QI", wall, logical) + b"\x0d"


def quoted_key(s: str) -> bytes:
    return s.encode("latin-1").decode("unicode_escape").encode("latin-1")


def parse_scan(lines, key_fn):
    out = []
    for ln in lines:
        m = re.match(r"^(.*)#(\d+),([A-Z]+) \[(.*)\]$", ln)
        assert m, ln
        k, seq, kind, val = m.groups()
        v = re.match(r"^\(f(\d+),blk(\d+),id(\d+),len(\d+)\)$", val)
        out.append({"key": key_fn(k).hex(), "seq": int(seq), "kind": KINDS[kind],
                    "value": None if v else val, "blob": [int(x) for x in v.groups()] if v else None})
    return out


def main():
    text = open(REF).read()
    blocks = text.split("\nsstable scan\n")
    res = {}
    for blk in blocks:
        head, _, body = blk.partition("\n----\n")
        args = head.strip().splitlines()
        if args == ["./testdata/cr-schema-sst/000014.sst"]:
            lines = [ln for ln in body.strip().splitlines()]
            assert lines[0] == "000014.sst"
            res["cr_schema_000014.sst"] = {"source": "tool/testdata/sstable_scan (sstable scan ./testdata/cr-schema-sst/000014.sst)",
                                           "kvs": parse_scan(lines[1:], crdb_key)}
        if args == ["./testdata/find-val-sep-db"]:
            cur = None
            for ln in body.strip().splitlines():
                m = re.match(r"^find-val-sep-db/(\d+)\.sst$", ln)
                if m:
                    cur = f"find_val_sep_{m.group(1)}.sst"
                    res[cur] = {"source": "tool/testdata/sstable_scan (sstable scan ./testdata/find-val-sep-db)",
                                "kvs": []}
                elif cur:
                    res[cur]["kvs"] += parse_scan([ln], quoted_key)
    assert len(res) == 4, sorted(res)
    json.dump(res, open(OUT, "w"), indent=1)
    print({k: len(v["kvs"]) for k, v in res.items()})


if __name__ == "__main__":
    main()
