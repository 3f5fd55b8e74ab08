"""Columnar tables through the device:
`Table(...).decode()` on the reference's Pebblev7 test tables reproduces its
`sstable scan` output (tool/testdata/sstable_scan:391-440) exactly -- metaindex
and properties as colblk KeyValueBlocks (pbl_kv_blocks), the key schema from
"pebble.colblk.schema", the two-level colblk index (AttributeTwoLevelIndex),
value blocks fetched on the device (pbl_valblk_index, pbl_resolve_values) and
blob handles kept as PBL_KV_BLOB_HANDLE values.  Each device step is also
checked against the oracle, with corrupt and overflowing inputs."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch
from pebble_amd.rowblk import kvs_of_block
from pebble_amd.sstable import KvSlices, Table, kv_blocks, resolve_values
from tableutil import TABLES, check_scan, table_bytes

pytestmark = pytest.mark.gpu


def table_kvs(r):
    out = []
    for b in range(len(r["blk_status"])):
        out += [(kv.user_key, kv.trailer, kv.value, kv.flags) for kv in kvs_of_block(r, b)]
    return out


@pytest.mark.parametrize("name", sorted(TABLES))
def test_table_decode_reproduces_sstable_scan(name):
    t = Table(table_bytes(name))
    assert t.key_schema() == N.PBL_FMT_COL_CRDB1
    r = t.decode().to_host()
    assert r["status_mask"] == 0
    kvs = table_kvs(r)
    check_scan(name, kvs)
    _props, okvs = oracle.table_scan(table_bytes(name))
    assert kvs == okvs


def test_metadata_matches_oracle():
    for name in TABLES:
        d = table_bytes(name)
        t = Table(d)
        props, _ = oracle.table_scan(d)
        assert t.properties() == props
        f = oracle.parse_footer(d[-61:], len(d))
        st, rows = oracle.kv_block_col(oracle.table_block(d, f["metaindex"]))
        assert st == 0
        assert t.metaindex() == {k: oracle.decode_handle(v, 0)[0] for k, v in rows}
    assert Table(table_bytes("cr_schema_000014.sst")).two_level()
    assert Table(table_bytes("find_val_sep_000011.sst")).two_level()
    assert not Table(table_bytes("find_val_sep_000005.sst")).two_level()


def test_unresolved_values_are_value_block_handles():
    t = Table(table_bytes("cr_schema_000014.sst"))
    kvs = table_kvs(t.decode(resolve=False).to_host())
    n_vb = sum(1 for _k, _t, _v, fl in kvs if fl & N.PBL_KV_VALBLK_HANDLE)
    assert n_vb > 0
    assert kvs[0][2].hex() == TABLES["cr_schema_000014.sst"]["kvs"][0]["value"]  # the in-place one


def test_two_level_attribute_mismatch_is_corruption():
    d = bytearray(table_bytes("find_val_sep_000011.sst"))
    t = Table(bytes(d))
    t.footer.attributes &= ~(1 << 5)
    with pytest.raises(Exception, match="attributes mismatch"):
        t.data_block_handles()


def pack(blocks, align=8):
    offs, lens, pos = [], [], 0
    for bk in blocks:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        lens.append(len(bk))
        pos += len(bk)
    buf = np.zeros(pos + 16, np.uint8)
    for o, bk in zip(offs, blocks):
        buf[o:o + len(bk)] = np.frombuffer(bk, np.uint8)
    return buf, np.array(offs, np.uint64), np.array(lens, np.uint32)


def test_kv_blocks_against_oracle():
    blocks = []
    for name in sorted(TABLES):
        d = table_bytes(name)
        f = oracle.parse_footer(d[-61:], len(d))
        meta = oracle.table_block(d, f["metaindex"])
        st, rows = oracle.kv_block_col(meta)
        blocks += [meta, oracle.table_block(d, oracle.decode_handle(dict(rows)[b"rocksdb.properties"], 0)[0])]
    bad = bytearray(blocks[0])
    bad[7] = 2
    blocks_all = blocks + [bytes(bad), blocks[1][:5]]
    for align in (8, 1):
        buf, off, lens = pack(blocks_all, align)
        kv = kv_blocks(BlockBatch.from_host(buf, off, lens, "cuda"))
        st = kv.status()
        base = kv.blk_base.cpu().numpy()
        ko, kl = kv.key_off.cpu().numpy(), kv.key_len.cpu().numpy()
        vo, vl = kv.val_off.cpu().numpy(), kv.val_len.cpu().numpy()
        raw = buf.tobytes()
        for i, blk in enumerate(blocks_all):
            ost, rows = oracle.kv_block_col(blk)
            assert st[i] == ost, i
            assert base[i + 1] - base[i] == len(rows)
            got = [(raw[ko[k]:ko[k] + kl[k]], raw[vo[k]:vo[k] + vl[k]]) for k in range(base[i], base[i + 1])]
            assert got == rows, i
    # capacity overflow: blocks that do not fit report PBL_OVERFLOW, the rest are written
    buf, off, lens = pack(blocks)
    bb = BlockBatch.from_host(buf, off, lens, "cuda")
    e = lambda n, dt: torch.empty(n, dtype=dt, device="cuda")  # noqa: E731
    out = KvSlices(e(20, torch.int64), e(20, torch.int32), e(20, torch.int64), e(20, torch.int32),
                   e(len(blocks) + 1, torch.int64), e(len(blocks), torch.int32))
    assert N.lib().pbl_kv_blocks(ctypes.byref(bb.c_struct()), ctypes.byref(out.c_struct()), None) == 0
    st = out.status()
    assert st[0] == 0 and (st == N.PBL_OVERFLOW).any()
    assert int(out.blk_base[len(blocks)].item()) > 20


def test_valblk_index_and_corrupt_handles():
    t = Table(table_bytes("cr_schema_000014.sst"))
    vb = t.value_blocks()
    assert vb is not None and vb.n_blocks >= 1
    d = t.decode(resolve=False)
    ok = resolve_values(d, vb).to_host()
    assert ok["status_mask"] == 0
    # every value block shortened to 1 byte: the handles run past their block
    short = BlockBatch(vb.blocks, vb.block_off, torch.ones_like(vb.block_len), vb.format, vb.flags)
    r = resolve_values(d, short).to_host()
    st = r["blk_status"]
    h = d.to_host()
    for b in range(len(st)):
        has_vb = any(kv.flags & N.PBL_KV_VALBLK_HANDLE for kv in kvs_of_block(h, b))
        assert st[b] == (N.PBL_CORRUPT_VALUE_HANDLE if has_vb else 0), b
    # no value blocks at all: every handle names a block past the batch
    empty = BlockBatch(vb.blocks, vb.block_off[:0], vb.block_len[:0], vb.format, vb.flags)
    r = resolve_values(d, empty).to_host()
    assert r["status_mask"] & (1 << N.PBL_CORRUPT_VALUE_HANDLE)
    # a value index whose block numbers are not in order is corrupt
    rows = np.array([[1, 0, 0, 10], [0, 0, 0, 20]], np.uint8)  # widths (1, 2, 1)
    src = torch.from_numpy(rows.reshape(-1).copy()).cuda()
    ho, hl = torch.empty(2, dtype=torch.int64, device="cuda"), torch.empty(2, dtype=torch.int64, device="cuda")
    n_st = torch.zeros(2, dtype=torch.int32, device="cuda")
    assert N.lib().pbl_valblk_index(src.data_ptr(), 8, 1, 2, 1, ho.data_ptr(), hl.data_ptr(), 2, n_st.data_ptr(),
                                    n_st.data_ptr() + 4, None) == 0
    assert n_st.cpu().tolist() == [2, N.PBL_CORRUPT_VALUE_HANDLE]
    rows[0, 0], rows[1, 0] = 0, 1
    src = torch.from_numpy(rows.reshape(-1).copy()).cuda()
    assert N.lib().pbl_valblk_index(src.data_ptr(), 8, 1, 2, 1, ho.data_ptr(), hl.data_ptr(), 2, n_st.data_ptr(),
                                    n_st.data_ptr() + 4, None) == 0
    torch.cuda.synchronize()
    assert n_st.cpu().tolist() == [2, 0] and hl.cpu().tolist() == [10, 20] and ho.cpu().tolist() == [0, 0]
