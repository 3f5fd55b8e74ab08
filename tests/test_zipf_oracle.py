"""Config 5 (BASELINE.json configs[4]): Zipf-skewed key lengths (8-1024 B) and
value lengths (0-64 KiB), restart interval 1/16/32 swept, row and colblk.
The generator's batches decode cleanly on the oracle (CPU, no GPU)."""
import numpy as np
import pytest

import oracle
from pebble_amd import _native as N
from pebble_amd.batch import gen_zipf_blocks


@pytest.mark.parametrize("ri", [1, 16, 32])
def test_zipf_row_blocks_decode_on_oracle(ri):
    buf, off, lens, n = gen_zipf_blocks(11 + ri, 96, N.PBL_FMT_ROW, ri)
    assert (off % 8 == 0).all() and (np.diff(off.astype(np.int64)) >= lens[:-1]).all()
    r = oracle.rowblk_decode_batch(buf, off, lens)
    assert r["status_mask"] == 0 and r["n_kv"] == n
    kl = np.diff(r["key_off"].astype(np.int64))
    vl = np.diff(r["val_off"].astype(np.int64))
    # per-block N+1 offsets: drop the block boundaries (negative / restart steps)
    kl, vl = kl[kl > 0], vl[vl >= 0]
    assert kl.min() >= 8 and kl.max() <= 1024  # user keys (the trailer is its own array)
    assert vl.max() <= 65536
    assert r["n_restarts"] >= -(-n // ri)
    # a block takes its first KV even when it alone exceeds the 32 KiB target
    big = lens > 32768
    assert (np.diff(r["blk_kv_base"].astype(np.int64))[big] == 1).all()


def test_zipf_col_blocks_decode_on_oracle():
    buf, off, lens, n = gen_zipf_blocks(5, 64, N.PBL_FMT_COL_DEFAULT)
    r = oracle.decode_batch(buf, off, lens, N.PBL_FMT_COL_DEFAULT)
    assert r["status_mask"] == 0 and r["n_kv"] == n
    assert r["val_bytes_total"] > 64 * 1024  # 32-bit RawBytes offsets are exercised


def test_zipf_generator_is_deterministic():
    a = gen_zipf_blocks(3, 16, N.PBL_FMT_ROW, 16)
    b = gen_zipf_blocks(3, 16, N.PBL_FMT_ROW, 16, n_threads=3)
    assert a[3] == b[3] and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_varlen_hint():
    """PBL_BATCH_VARLEN (a scheduling hint) is set for config 5's Zipf-sized
    blocks and not for fixed-size batches (configs 2/3)."""
    from pebble_amd.batch import varlen_hint
    assert varlen_hint(np.full(100, 32768, np.uint32)) == 0
    assert varlen_hint(np.r_[np.full(50, 8000), np.full(50, 60000)]) == N.PBL_BATCH_VARLEN
    _, _, lens, _ = gen_zipf_blocks(7, 200, N.PBL_FMT_COL_DEFAULT)
    assert varlen_hint(lens) == N.PBL_BATCH_VARLEN


def test_varlen_hint_row_density():
    """With the host bytes of a row batch the hint also samples the blocks'
    entry counts: value-dominated Zipf blocks keep PBL_BATCH_VARLEN (the
    two-pass row form), a mix of config-2 blocks and short table tails (many
    small KVs per block) does not (the pool kernel)."""
    from pebble_amd.batch import _row_entries, gen_row_mix, varlen_hint
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, n = gen_zipf_blocks(8, 200, N.PBL_FMT_ROW, 16)
    assert varlen_hint(lens, buf, off, N.PBL_FMT_ROW) == N.PBL_BATCH_VARLEN
    assert varlen_hint(lens, buf, off, N.PBL_FMT_COL_DEFAULT) == N.PBL_BATCH_VARLEN  # (only row batches sample)
    assert sum(_row_entries(bytes(buf[o:o + l])) for o, l in zip(off, lens)) == n
    buf, off, lens, n = gen_row_mix(9, 200, "tail8")
    assert varlen_hint(lens) == N.PBL_BATCH_VARLEN
    assert varlen_hint(lens, buf, off, N.PBL_FMT_ROW) == 0
    b2, o2, l2, n2 = gen_row_blocks(3, 4, 32768, 16, 16, 100)
    assert _row_entries(bytes(b2[o2[0]:o2[0] + l2[0]])) == n2 // 4
    assert _row_entries(b"\x00\x01") == -1
