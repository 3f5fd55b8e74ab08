"""The blockiter.Data adapter over a batch decoded ON THE DEVICE: the
reference's crdb1 table (cockroachkvs.Comparer) and config-2 row blocks
(DefaultComparer),
every block walked forward and backward and every key sought, the KVs equal to
the decoded arrays (pebble_amd/csrc/data_iter.cpp over DecodedBatch.to_host())."""
import random

import numpy as np
import pytest

from pebble_amd import _native as N
from pebble_amd.batch import BlockBatch, decode
from pebble_amd.blockiter import DataIter, key_compare

pytestmark = pytest.mark.gpu


def _walk(h, b, comparer):
    it = DataIter(h, b, comparer)
    assert it.status == 0
    kv0, kv1 = int(h["blk_kv_base"][b]), int(h["blk_kv_base"][b + 1])
    ko = h["key_off"][kv0 + b: kv1 + b + 1].astype(np.int64)
    kbase = int(h["blk_key_base"][b])
    keys = [h["key_bytes"][kbase + ko[j]: kbase + ko[j + 1]].tobytes() for j in range(kv1 - kv0)]
    fwd, kv = [], it.First()
    while kv is not None:
        fwd.append(kv.user_key)
        kv = it.Next()
    assert fwd == keys
    bwd, kv = [], it.Last()
    while kv is not None:
        bwd.append(kv.user_key)
        kv = it.Prev()
    assert bwd == keys[::-1]
    for a, c in zip(keys, keys[1:]):
        assert key_compare(comparer, a, c) <= 0
    rng = random.Random(b)
    for j in rng.sample(range(len(keys)), min(len(keys), 20)):
        first = next(i for i in range(len(keys)) if key_compare(comparer, keys[i], keys[j]) >= 0)
        assert it.SeekGE(keys[j]).user_key == keys[first]
        assert int(it.KV().trailer) == int(h["trailer"][kv0 + first])


def test_adapter_over_the_reference_crdb1_table():
    # cr-schema-sst/000014.sst (CockroachDB keys, crdb1 colblk) decoded on the device
    from pebble_amd.sstable import Table
    from tableutil import table_bytes
    h = Table(table_bytes("cr_schema_000014.sst")).decode().to_host()
    assert h["status_mask"] == 0
    for b in range(len(h["blk_status"])):
        _walk(h, b, N.PBL_CMP_CRDB)


def test_adapter_over_device_decoded_row_blocks():
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, n = gen_row_blocks(8, 64, 32768, 16, 16, 100, n_threads=4)
    h = decode(BlockBatch.from_host(buf, off, lens, "cuda", N.PBL_FMT_ROW, 0)).to_host()
    for b in range(0, 64, 9):
        _walk(h, b, N.PBL_CMP_DEFAULT)
