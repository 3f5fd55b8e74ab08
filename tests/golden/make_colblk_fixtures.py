#!/usr/bin/env python3
"""Columnar (colblk) golden fixtures, read as DATA from the reference's own
datadriven test files (run in the container that has /root/reference; the GPU
box only reads the generated tests/golden/colblk_golden.json).

Every case is a whole serialized data block, recovered byte-for-byte from the
`describe`/`finish`/`rewrite` hex dumps the reference's tests print
(binfmt lines `NNN-MMM: x HEX` / `b BITS`), together with the KVs the
reference's test wrote into that block:

  sstable/colblk/testdata/data_block/*   DefaultKeySchema(testkeys.Comparer, bundle)
        writer input:  `write` lines, parsed as data_block_test.go:76-109 does
        (value-handle / blob-handle prefixes, obsolete marking, PrefixEqual)
  cockroachkvs/testdata/block_encoding   cockroachkvs.KeySchema ("crdb1")
        writer input:  the `init` lines; expected decode: the `keys` output
        (cockroachkvs_test.go formatUserKey: `roachKey @ HEXVERSION #seq,KIND = value`)
  sstable/testdata/writer_tiering_histogram   Pebblev8 blocks with the tiering columns
        (`layout` dumps; tiering_cases below), plus the tiering KV/meta KATs

The expected per-row output is derived from the writer input alone (never from
the dump), so a decoder that reproduces it from the dumped bytes is pinned to
the reference's own encoder.
"""
from __future__ import annotations

import ast
import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

KINDS = {"DEL": 0, "SET": 1, "MERGE": 2, "LOGDATA": 3, "SINGLEDEL": 7, "RANGEDEL": 15, "SEPARATOR": 17,
         "SETWITHDEL": 18, "RANGEKEYDEL": 19, "RANGEKEYUNSET": 20, "RANGEKEYSET": 21, "INGESTSST": 22,
         "DELSIZED": 23, "EXCISE": 24, "SYNTHETIC": 25, "INGESTSSTWITHBLOB": 26, "BDRY": 30, "INVALID": 191}
# internal/base/internal.go:97-217 ; trailer = seq<<8 | kind (internal.go:279-314)
SEQ_MAX = (1 << 56) - 1

LINE = re.compile(r"(\d+)-(\d+): ([xb])((?: [0-9a-f]+)*)")


def parse_datadriven(path: str):
    sys.path.insert(0, HERE)
    from make_fixtures import parse_datadriven as pdd  # same file format as the rowblk fixtures
    lines = open(path).read().split("\n")
    cases = pdd(path)
    # attach source line numbers (first occurrence of each command line, in order)
    pos = 0
    for c in cases:
        while pos < len(lines) and lines[pos] != c["cmd"]:
            pos += 1
        c["line"] = pos + 1
        pos += 1
    return cases


def dump_to_bytes(text: str) -> bytes:
    """Rebuild a block from binfmt lines; every byte must be covered exactly once."""
    spans = []
    for m in LINE.finditer(text):
        a, b, kind, payload = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4).replace(" ", "")
        if kind == "x":
            data = bytes.fromhex(payload)
        else:
            assert len(payload) % 8 == 0, payload
            data = bytes(int(payload[i:i + 8], 2) for i in range(0, len(payload), 8))
        assert len(data) == b - a, (a, b, payload)
        spans.append((a, data))
    n = max(a + len(d) for a, d in spans)
    out = bytearray(n)
    cov = bytearray(n)
    for a, d in spans:
        out[a:a + len(d)] = d
        for i in range(a, a + len(d)):
            cov[i] += 1
    assert all(c == 1 for c in cov), "hex dump does not cover the block exactly once"
    return bytes(out)


def parse_ikey(s: str):
    """base.ParseInternalKey (internal/base/internal.go:616-630)."""
    i, j = s.index("#"), s.index(",")
    seq = int(s[i + 1:j])
    return s[:i].encode(), (seq << 8) | KINDS[s[j + 1:]]


def testkeys_split(k: bytes) -> int:
    """testkeys.Comparer.Split: prefix is everything before the last '@'
    (internal/testkeys/testkeys.go:144-150)."""
    i = k.rfind(b"@")
    return len(k) if i < 0 else i


def default_schema_rows(write_lines):
    """data_block_test.go:76-109 -> the rows the encoder saw."""
    rows, prev_key, prev_kind = [], None, None
    for line in write_lines:
        obsolete = False
        if line.endswith("obsolete"):
            line, obsolete = line[: -len("obsolete")], True
        j = line.index(":")
        ukey, trailer = parse_ikey(line[:j])
        value = line[j + 1:].encode()
        prefix_equal = prev_key is not None and prev_key[:testkeys_split(prev_key)] == ukey[:testkeys_split(ukey)]
        vp = None  # in place
        if value.startswith(b"valueHandle"):
            vp = 0x80 | (0x20 if prefix_equal else 0)   # block.ValueBlockHandlePrefix(prefixEqual, 0)
        elif value.startswith(b"blobHandle"):
            vp = 0x40 | (0x20 if prefix_equal else 0)   # block.BlobValueHandlePrefix(prefixEqual, 0)
        if prev_key == ukey and prev_kind != 2:
            obsolete = True
        stored = value if vp is None else bytes([vp]) + value
        rows.append({"key": ukey.hex(), "trailer": trailer, "value": stored.hex(), "raw_value": value.hex(),
                     "vp": -1 if vp is None else vp, "external": vp is not None, "obsolete": obsolete,
                     "prefix_changed": not prefix_equal, "prefix_len": testkeys_split(ukey)})
        prev_key, prev_kind = ukey, trailer & 0xFF
    return rows


def data_block_cases():
    out = []
    d = os.path.join(REF, "sstable/colblk/testdata/data_block")
    for fn in sorted(os.listdir(d)):
        path = os.path.join(d, fn)
        rel = os.path.relpath(path, REF)
        bundle, written, finished = 16, [], None
        for c in parse_datadriven(path):
            cmd = c["cmd"].split()
            if cmd[0] == "init":
                bundle, written = 16, []
                for a in cmd[1:]:
                    if a.startswith("bundle-size="):
                        bundle = int(a.split("=")[1])
            elif cmd[0] == "write-block":
                bundle, written, finished = 16, default_schema_rows([l for l in c["input"].split("\n") if l]), None
            elif cmd[0] == "write":
                written = written + [l for l in c["input"].split("\n") if l]
            elif cmd[0] == "finish":
                nrows = len(written)
                for a in cmd[1:]:
                    if a.startswith("rows="):
                        nrows = int(a.split("=")[1])
                all_rows = default_schema_rows(written)
                rows = all_rows[:nrows]
                blk = dump_to_bytes(c["expected"])
                finished = (rows, blk)
                out.append({"name": f"{fn}:{c['line']}", "source": f"{rel}:{c['line']}", "schema": "default",
                            "bundle_size": bundle, "block": blk.hex(), "rows": rows, "encoder_exact": True,
                            "writer_rows": all_rows, "finish_rows": nrows})
            elif cmd[0] == "rewrite" and not c["expected"].startswith("error"):
                frm = to = None
                for a in cmd[1:]:
                    if a.startswith("from="):
                        frm = a.split("=", 1)[1].encode()
                    if a.startswith("to="):
                        to = a.split("=", 1)[1].encode()
                rows = []
                for r in finished[0]:
                    k = bytes.fromhex(r["key"])
                    p = testkeys_split(k)
                    assert k[p:] == frm, (k, frm)
                    rows.append(dict(r, key=(k[:p] + to).hex()))
                blk = dump_to_bytes(c["expected"])
                out.append({"name": f"{fn}:{c['line']}", "source": f"{rel}:{c['line']}", "schema": "default",
                            "bundle_size": bundle, "block": blk.hex(), "rows": rows, "encoder_exact": False})
    return out


def go_unquote(s: str) -> bytes:
    if s.startswith('"'):
        return ast.literal_eval("b" + s)
    return s.encode()


def crdb_key(text: str):
    """`roachKey [@ HEXVERSION] #seq,KIND = value` -> (user key, trailer, value)
    (cockroachkvs_test.go parseUserKey / formatUserKey; cockroachkvs.go:140-309)."""
    kpart, value = text.split(" = ", 1)
    kpart, ik = kpart.rsplit(" #", 1)
    seq, kind = ik.split(",")
    if " @ " in kpart:
        roach, ver = kpart.split(" @ ")
        ver = bytes.fromhex(ver)
    else:
        roach, ver = kpart, b""
    key = go_unquote(roach.strip()) + b"\x00"
    if ver:
        key += ver + bytes([len(ver) + 1])
    return key, (int(seq) << 8) | KINDS[kind], value.encode()


def crdb1_cases():
    path = os.path.join(REF, "cockroachkvs/testdata/block_encoding")
    rel = os.path.relpath(path, REF)
    cases = parse_datadriven(path)
    init = next(c for c in cases if c["cmd"].startswith("init"))
    keys = next(c for c in cases if c["cmd"].startswith("keys"))
    desc = next(c for c in cases if c["cmd"].startswith("describe"))
    inp = [crdb_key(l) for l in init["input"].split("\n") if l]
    exp = [crdb_key(l) for l in keys["expected"].split("\n") if l]
    assert len(inp) == len(exp)
    rows, prev = [], None
    for (ik, it, iv), (ek, et, ev) in zip(inp, exp):
        assert it == et and iv == ev
        roach_len = len(ik) - (ik[-1] if ik[-1] != 0 else 0)  # roach key + sentinel
        pc = prev is None or prev != ik[:roach_len]
        rows.append({"key": ek.hex(), "in_key": ik.hex(), "trailer": et, "value": ev.hex(), "raw_value": iv.hex(),
                     "vp": -1, "external": False, "obsolete": False, "prefix_changed": pc, "prefix_len": roach_len})
        prev = ik[:roach_len]
    blk = dump_to_bytes(desc["expected"])
    return [{"name": f"block_encoding:{desc['line']}", "source": f"{rel}:{init['line']}-{desc['line']}",
             "schema": "crdb1", "bundle_size": 16, "block": blk.hex(), "rows": rows, "encoder_exact": True,
             "writer_rows": [dict(r, key=r["in_key"]) for r in rows], "finish_rows": len(rows)}]


def _args(cmd: str) -> dict:
    out = {}
    for tok in cmd.split()[1:]:
        k, _, v = tok.partition("=")
        out[k] = v if v else True
    return out


def codec_cases():
    """Per-codec dumps (uints, raw_bytes, prefix_bytes, bitmap) recorded
    verbatim, each with the values a decoder must return, derived from the
    reference test's own inputs (never from the dump):
      uints         the `write i:v` lines since the last `init` (unwritten rows 0)
                    (uints_test.go TestUints)
      raw_bytes     the `build` input lines (first `count=` of them)
                    (raw_bytes_test.go)
      prefix_bytes  the keys `put` since the last `init` (first `rows=` of them)
                    (prefix_bytes_test.go; `get`/`unsafe-get` print the same keys)
      bitmap        the bit string the reference's own DecodeBitmap printed (the
                    lines before "Binary representation:") (bitmap_test.go:25-70)
    `offset` is where the column starts in the bytes."""
    out = {}
    for fn in ("uints", "raw_bytes", "prefix_bytes", "bitmap"):
        path = os.path.join(REF, "sstable/colblk/testdata", fn)
        rel = os.path.relpath(path, REF)
        lst = []
        writes, puts = {}, []
        for c in parse_datadriven(path):
            a = _args(c["cmd"])
            verb = c["cmd"].split()[0]
            if verb == "init":
                writes, puts = {}, []
            elif verb == "write":
                for f in c["input"].split():
                    i, v = f.split(":")
                    writes[int(i)] = int(v)
            elif verb == "put":
                puts += [k for k in c["input"].strip().split("\n")]
            if not (LINE.search(c["expected"]) and not c["expected"].startswith("error")):
                continue
            try:
                blk = dump_to_bytes(c["expected"])
            except AssertionError:
                continue
            e = {"source": f"{rel}:{c['line']}", "cmd": c["cmd"], "input": c["input"], "bytes": blk.hex(),
                 "dump": c["expected"], "offset": int(a.get("offset", 0))}
            if fn == "uints" and verb == "finish":
                rows = int(a["rows"])
                e.update(rows=rows, expect=[writes.get(i, 0) for i in range(rows)])
            elif fn == "raw_bytes" and verb == "build":
                sl = c["input"].split("\n")
                if "count" in a:
                    sl = sl[: int(a["count"])]
                e.update(rows=len(sl), expect=[x.encode().hex() for x in sl])
            elif fn == "prefix_bytes" and verb == "finish":
                rows = int(a["rows"])
                e.update(rows=rows, expect=[k.encode().hex() for k in puts[:rows]])
            elif fn == "bitmap" and verb == "build":
                bits = "".join(c["expected"].split("Binary representation:")[0].split())
                e.update(rows=len(bits), expect=[int(ch) for ch in bits])
            lst.append(e)
        out[fn] = lst
    return out


ITER_LINE = re.compile(r"^\s*(first|next):\s*(.*)$")


def transform_cases():
    """sstable/colblk/testdata/data_block/transforms: each `write-block` (rows
    the DataBlockEncoder saw, data_block_test.go:76-109) with the `iter <args>`
    cases run over it (args: synthetic-seq-num, hide-obsolete-points,
    synthetic-prefix, synthetic-suffix; data_block_test.go:140-160).  Kept: the
    forward scan each case prints from `first` through its consecutive `next`
    commands, as (user key, seq or None, kind or None, value) rows; None after
    the last row = the iterator was exhausted ('.')."""
    path = os.path.join(REF, "sstable/colblk/testdata/data_block/transforms")
    rel = os.path.relpath(path, REF)
    out, rows = [], None
    for c in parse_datadriven(path):
        cmd = c["cmd"].split()
        if cmd[0] == "write-block":
            rows = default_schema_rows([l for l in c["input"].split("\n") if l])
            out.append({"source": f"{rel}:{c['line']}", "rows": rows, "iters": []})
        elif cmd[0] == "iter":
            cmds = [l.strip() for l in c["input"].split("\n") if l.strip()]
            if not cmds or cmds[0] != "first":
                continue
            n = 1
            while n < len(cmds) and cmds[n] == "next":
                n += 1
            seq = []
            for line in c["expected"].split("\n")[:n]:
                m = ITER_LINE.match(line)
                assert m, line
                body = m.group(2).strip()
                if body == ".":
                    seq.append(None)
                    break
                k, _, v = body.partition(":")
                if "#" in k:
                    uk, tr = parse_ikey(k)
                    seq.append([uk.hex(), tr >> 8, tr & 0xFF, v.encode().hex()])
                else:
                    seq.append([k.encode().hex(), None, None, v.encode().hex()])
            args = _args(c["cmd"])
            out[-1]["iters"].append({"line": c["line"], "seq_num": int(args.get("synthetic-seq-num", 0)),
                                     "hide_obsolete": bool(args.get("hide-obsolete-points", False)),
                                     "prefix": str(args.get("synthetic-prefix", "")).encode().hex(),
                                     "suffix": str(args.get("synthetic-suffix", "")).encode().hex(),
                                     "forward": seq})
    return out


TIER = re.compile(r";tiering:span=(\d+),attr=(\d+)$")


def _tier_meta(value: str):
    """testkeys.ExtractKVMeta (sstable/test_utils.go:182-186): a value ending in
    ";tiering:span=S,attr=A" carries KVMeta{S, A}; the value keeps the text."""
    m = TIER.search(value)
    return (int(m.group(1)), int(m.group(2))) if m else (0, 0)


def _layout_data_blocks(text: str):
    """The `data` entries of a `layout` dump: (hex-dump text, KV lines) each."""
    out, cur = [], None
    for line in text.split("\n"):
        if line.startswith(" ├── data ") or line.startswith(" └── data "):
            cur = {"dump": [], "kvs": []}
            out.append(cur)
            continue
        if line.startswith(" ├── ") or line.startswith(" └── "):
            cur = None
            continue
        if cur is None:
            continue
        if LINE.search(line):
            cur["dump"].append(line)
        else:
            m = re.match(r"^ │    [├└]── (\S.*)$", line)
            if m and "#" in m.group(1) and not m.group(1).startswith("trailer"):
                cur["kvs"].append(m.group(1))
    return [("\n".join(b["dump"]), b["kvs"]) for b in out]


def tiering_cases():
    """Pebblev8 data blocks with the tiering columns (sstable/format.go:305-316;
    data_block.go:514-525), recovered byte-for-byte from the only whole-block
    dumps of that layout the reference holds: the `layout` outputs of
    sstable/testdata/writer_tiering_histogram (DefaultKeySchema(testkeys, 16),
    writer input from the preceding `build`).  Expected rows come from the
    writer input: key and trailer, the value (in place: the input text; a
    dual-tier blob value: the dumped column slice, isValueExternal), and the
    KVMeta the writer stored (ExtractKVMeta; KVMeta{} without a tiering suffix).
    Also the KV + meta KATs with no dump: colblk/data_block_meta_test.go:27-33
    (TestDataBlockIterWithMeta) and the `build` / `scan-compaction` pair of
    sstable/testdata/writer_v8:388-402 (NextWithMeta's output)."""
    path = os.path.join(REF, "sstable/testdata/writer_tiering_histogram")
    rel = os.path.relpath(path, REF)
    blocks, build = [], None
    for c in parse_datadriven(path):
        verb = c["cmd"].split()[0]
        if verb == "build":
            build = c
        elif verb == "layout" and "data for column" in c["expected"]:
            lines = [l for l in build["input"].split("\n") if l]
            for dump, kv_lines in _layout_data_blocks(c["expected"]):
                blk = dump_to_bytes(dump)
                rows, prev = [], None
                exact = True
                for i, line in enumerate(lines[: len(kv_lines)]):
                    j = line.index(":")
                    ukey, trailer = parse_ikey(line[:j])
                    text = line[j + 1:]
                    pl = testkeys_split(ukey)
                    row = {"key": ukey.hex(), "trailer": trailer, "obsolete": False, "prefix_len": pl,
                           "prefix_changed": prev is None or prev[:testkeys_split(prev)] != ukey[:pl]}
                    if text.startswith("hot-blob{"):
                        exact = False
                        row.update(value=None, external=True, span=0, attr=0, dump_value=True)
                    else:
                        sp, at = _tier_meta(text)
                        row.update(value=text.encode().hex(), external=False, span=sp, attr=at, vp=-1)
                    rows.append(row)
                    prev = ukey
                blocks.append({"name": f"writer_tiering_histogram:{c['line']}", "source": f"{rel}:{build['line']}-{c['line']}",
                               "schema": "default", "bundle_size": 16, "block": blk.hex(), "rows": rows,
                               "encoder_exact": exact})
    kats = [{"source": "sstable/colblk/data_block_meta_test.go:27-33", "schema": "default", "bundle_size": 16,
             "kvs": [["a#1,SET", "value", 42, 100], ["b#2,SET", "value", 43, 200], ["c#3,SET", "value", 0, 0]]}]
    path = os.path.join(REF, "sstable/testdata/writer_v8")
    rel = os.path.relpath(path, REF)
    build = None
    for c in parse_datadriven(path):
        verb = c["cmd"].split()[0]
        if verb == "build":
            build = c
        elif verb == "scan-compaction":
            kvs = []
            for line in c["expected"].split("\n"):
                if not line:
                    continue
                kv, _, meta = line.rpartition(" meta=")
                j = kv.index(":")
                if meta == "<no meta>":
                    sp, at = 0, 0
                else:
                    m = re.fullmatch(r"tiering:span=(\d+),attr=(\d+)", meta)
                    sp, at = int(m.group(1)), int(m.group(2))
                kvs.append([kv[:j], kv[j + 1:], sp, at])
            inp = [l for l in build["input"].split("\n") if l]
            assert [k[0] + ":" + k[1] for k in kvs] == inp
            kats.append({"source": f"{rel}:{build['line']}-{c['line']}", "schema": "default", "bundle_size": 16,
                         "kvs": kvs})
    return {"blocks": blocks, "kats": kats}


def main():
    cases = data_block_cases() + crdb1_cases()
    res = {"data_blocks": cases, "codecs": codec_cases(), "transforms": transform_cases(),
           "tiering": tiering_cases()}
    p = os.path.join(HERE, "colblk_golden.json")
    with open(p, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", p, len(cases), "data blocks,", {k: len(v) for k, v in res["codecs"].items()}, "codec dumps,",
          sum(len(t["iters"]) for t in res["transforms"]), "transform scans,",
          len(res["tiering"]["blocks"]), "tiering blocks,", len(res["tiering"]["kats"]), "tiering KATs")


if __name__ == "__main__":
    main()
