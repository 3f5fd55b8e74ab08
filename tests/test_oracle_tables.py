"""Columnar tables, CPU side: the oracle's whole-table walk
-- KeyValueBlock metaindex and properties, two-level colblk index, key schema
from "pebble.colblk.schema", value blocks -- reproduces the reference's own
`sstable scan` output for its Pebblev7 test tables (tool/testdata/sstable_scan
:391-440): cockroach-schema 000014.sst (two-level index, values in value
blocks) and the find-val-sep-db tables (blob handles)."""
import pytest

import oracle
from tableutil import TABLES, check_scan, table_bytes


@pytest.mark.parametrize("name", sorted(TABLES))
def test_oracle_table_scan_matches_sstable_scan(name):
    props, kvs = oracle.table_scan(table_bytes(name))
    assert props[b"pebble.colblk.schema"] == b"crdb1"
    check_scan(name, kvs)


def test_fixture_attributes():
    """The footers' attribute bits agree with the properties (reader.go:1214-1221):
    000014 and 000011 are two-level, 000014 has value blocks, the others blob values."""
    for name, two, vb, blob in [("cr_schema_000014.sst", 1, 1, 0), ("find_val_sep_000005.sst", 0, 0, 1),
                                ("find_val_sep_000011.sst", 1, 0, 1)]:
        d = table_bytes(name)
        f = oracle.parse_footer(d[-61:], len(d))
        a = f["attributes"]
        assert (bool(a & 1 << 5), bool(a & 1), bool(a & 1 << 6)) == (bool(two), bool(vb), bool(blob)), name
        props, _ = oracle.table_scan(d)
        assert int.from_bytes(props[b"rocksdb.block.based.table.index.type"], "little") == (2 if two else 0)


def test_kv_block_col_rejects_malformed_columns():
    d = table_bytes("cr_schema_000014.sst")
    f = oracle.parse_footer(d[-61:], len(d))
    blk = oracle.table_block(d, f["metaindex"])
    st, rows = oracle.kv_block_col(blk)
    assert st == 0 and b"rocksdb.properties" in dict(rows)
    bad = bytearray(blk)
    bad[7] = 2  # column 0 claims uints
    assert oracle.kv_block_col(bytes(bad))[0] == 4
    assert oracle.kv_block_col(blk[:6])[0] == 4
