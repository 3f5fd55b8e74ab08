"""Config 5 (BASELINE.json configs[4]) on the GPU: Zipf-skewed key lengths
(8-1024 B) and values (0-64 KiB), restart interval 1/16/32 swept; row, colblk
(DefaultKeySchema) and mixed batches.  Bit-exact against the oracle on every
output array; blocks past the LDS stage take the general path, which must agree
too."""
import numpy as np
import pytest

from pebble_amd import _native as N
from pebble_amd.batch import gen_zipf_blocks
from test_colblk_gpu import check as col_check
from test_rowblk_gpu import check as row_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ri", [1, 16, 32])
@pytest.mark.parametrize("vp", [False, True])
def test_zipf_row(ri, vp):
    buf, off, lens, n = gen_zipf_blocks(100 + ri, 400, N.PBL_FMT_ROW, ri)
    # vp: the blocks carry no value prefix, so reading them as prefixed must
    # fail the same blocks in the same way as the oracle (empty SET values)
    g = row_check(buf, off, lens, N.PBL_ROW_VALUE_PREFIX if vp else 0, f"zipf row ri={ri} vp={vp}")
    if not vp:
        assert g["n_kv"] == n and g["status_mask"] == 0
        assert g["n_slow_blocks"] >= int((lens > 32768).sum())
    # the row kernel must route every block past the 32 KiB stage to the
    # big-block passes (the count may be larger: blocks on the general walk)
    for kern in (N.PBL_KERNEL_POOL,):
        g = row_check(buf, off, lens, (N.PBL_ROW_VALUE_PREFIX if vp else 0) | kern, f"zipf row ri={ri} vp={vp} k={kern:#x}")
        if not vp:
            assert g["n_slow_blocks"] >= int((lens > 32768).sum())


@pytest.mark.parametrize("seed", [7, 8, 9])
@pytest.mark.parametrize("kernel", ["auto", "pipe"])
def test_zipf_col(seed, kernel):
    # auto: the batch carries PBL_BATCH_VARLEN -> the two-pass wave form (8 KiB stage);
    # pipe: the persistent pipeline forced on the same blocks (PBL_KERNEL_PIPE)
    buf, off, lens, n = gen_zipf_blocks(seed, 400, N.PBL_FMT_COL_DEFAULT)
    g = col_check(buf, off, lens, N.PBL_FMT_COL_DEFAULT, ctx="zipf col",
                  flags=N.PBL_KERNEL_PIPE if kernel == "pipe" else 0)
    assert g["n_kv"] == n


def test_zipf_mixed():
    rb, ro, rl, rn = gen_zipf_blocks(21, 200, N.PBL_FMT_ROW, 16)
    cb, co, cl, cn = gen_zipf_blocks(22, 200, N.PBL_FMT_COL_DEFAULT)
    rend = int(ro[-1]) + int(rl[-1] + 7) // 8 * 8
    buf = np.concatenate([rb[:rend], cb])
    off = np.concatenate([ro, co + rend]).astype(np.uint64)
    lens = np.concatenate([rl, cl]).astype(np.uint32)
    perm = np.random.default_rng(5).permutation(400)
    fmt = np.array([N.PBL_FMT_ROW] * 200 + [N.PBL_FMT_COL_DEFAULT] * 200, np.uint8)
    g = col_check(buf, off[perm].copy(), lens[perm].copy(), N.PBL_FMT_ROW, fmt[perm].copy(), ctx="zipf mixed")
    assert g["n_kv"] == rn + cn
