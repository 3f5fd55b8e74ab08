"""The PCIe-inclusive host pipeline (pebble_amd/pipeline.py): every chunk's
host arrays equal the oracle's decode of that chunk's blocks, for row, colblk
and mixed batches, ragged (variable-length, unaligned) layouts and a final
partial chunk."""
import numpy as np
import pytest
import torch

import oracle
from pebble_amd import _native as N
from pebble_amd.batch import Capacity
from pebble_amd.pipeline import stream_batch

pytestmark = pytest.mark.gpu


def check(buf, off, lens, fmt, block_fmt=None, chunk=64):
    host = torch.from_numpy(np.ascontiguousarray(buf)).pin_memory()
    o = oracle.decode_batch(buf, off, lens, fmt, block_fmt)
    cap = Capacity(o["n_kv"], o["key_bytes_total"], o["val_bytes_total"], o["n_restarts"])
    outs, _, pipe = stream_batch(host, off, lens, fmt, 0, cap, "cuda", chunk_blocks=chunk, block_format=block_fmt)
    assert len(outs.chunks) == (len(off) + chunk - 1) // chunk
    for c, ch in enumerate(outs.chunks):
        b0, b1 = ch.first_block, ch.first_block + ch.n_blocks
        oc = oracle.decode_batch(buf, off[b0:b1], lens[b0:b1], fmt,
                                 None if block_fmt is None else block_fmt[b0:b1])
        assert ch.status_mask == 0 and ch.n_kv == oc["n_kv"]
        for name, dt in (("trailer", np.uint64), ("kv_flags", np.uint8), ("key_off", np.uint32),
                         ("val_off", np.uint32), ("key_bytes", np.uint8), ("val_bytes", np.uint8)):
            assert np.array_equal(outs.view(c, name, dt), oc[name]), (c, name)
    # a second pass through the same pipeline gives the same bytes
    outs2, _, _ = stream_batch(host, off, lens, fmt, 0, cap, "cuda", chunk_blocks=chunk, pipe=pipe,
                               block_format=block_fmt)
    assert [c.n_kv for c in outs2.chunks] == [c.n_kv for c in outs.chunks]


def test_row_chunks():
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, _ = gen_row_blocks(3, 300, 4096, 16, 16, 100)
    check(buf, off, lens, N.PBL_FMT_ROW)


def test_col_chunks_ragged():
    from pebble_amd.colblk import gen_col_blocks
    buf, off, lens, _ = gen_col_blocks(4, 200, 8192)
    # repack at ragged offsets (8-B aligned and not)
    rng = np.random.default_rng(1)
    pos, offs, parts = 0, [], []
    for o, l in zip(off, lens):
        pos += int(rng.integers(0, 24))
        offs.append(pos)
        parts.append((pos, buf[int(o):int(o) + int(l)]))
        pos += int(l)
    nbuf = np.zeros(pos + 16, np.uint8)
    for p, b in parts:
        nbuf[p:p + len(b)] = b
    check(nbuf, np.array(offs, np.uint64), lens, N.PBL_FMT_COL_CRDB1, chunk=48)


def test_mixed_chunks():
    from pebble_amd.colblk import gen_col_blocks
    from pebble_amd.rowblk import gen_row_blocks
    rb, ro, rl, _ = gen_row_blocks(5, 100, 8192, 16, 16, 100)
    cb, co, cl, _ = gen_col_blocks(6, 100, 8192)
    buf = np.concatenate([rb[: int(ro[-1] + rl[-1])], np.zeros(8, np.uint8), cb])
    base = int(ro[-1] + rl[-1]) + 8
    off = np.empty(200, np.uint64)
    lens = np.empty(200, np.uint32)
    bf = np.empty(200, np.uint8)
    off[0::2], off[1::2] = ro, co + np.uint64(base)
    lens[0::2], lens[1::2] = rl, cl
    bf[0::2], bf[1::2] = N.PBL_FMT_ROW, N.PBL_FMT_COL_CRDB1
    check(buf, off, lens, N.PBL_FMT_ROW, bf, chunk=64)
