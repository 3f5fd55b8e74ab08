"""The RCCL branch of the offset concat (pebble_amd/shard.py allgather_totals,
backend "nccl"), executed for real: a world-size-1 `nccl` process group on the
one GPU, ShardedBatchDecoder.decode() with its default gather, against the
oracle -- plus the same all-gather + rebase bench.py's N > 1 step performs
(concat_step over all_gather_into_tensor of device tensors).  SURVEY.md §8(e):
blocks are independent (rowblk_iter.go:241-276), the only exchange is the
all-gather of the per-rank totals."""
import os
import socket

import numpy as np
import pytest

import oracle
from pebble_amd import _native as N
from pebble_amd.colblk import gen_col_blocks
from pebble_amd.rowblk import gen_row_blocks
from test_rowblk_gpu import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["row", "col", "mixed"])
def test_sharded_decoder_over_rccl(nccl_group, kind):
    import torch
    from pebble_amd.shard import ShardedBatchDecoder, allgather_totals
    fmt, bf = N.PBL_FMT_ROW, None
    if kind == "row":
        buf, off, lens, _ = gen_row_blocks(31, 256, 32768, 16, 16, 100)
    elif kind == "col":
        buf, off, lens, _ = gen_col_blocks(31, 256)
        fmt = N.PBL_FMT_COL_CRDB1
    else:
        rb, ro, rl, _ = gen_row_blocks(32, 128, 16384, 16, 16, 100)
        cb, co, cl, _ = gen_col_blocks(32, 128, 16384)
        buf = np.concatenate([rb[:128 * 16384], cb])
        off = np.concatenate([ro, co + np.uint64(128 * 16384)]).astype(np.uint64)
        lens = np.concatenate([rl, cl]).astype(np.uint32)
        bf = np.array([0] * 128 + [2] * 128, np.uint8)
    sd = ShardedBatchDecoder(buf, off, lens, fmt, 0, block_format=bf)  # rank / world from the nccl group
    assert sd.world == 1 and sd.block_range == (0, len(off))
    out, gathered = sd.decode()  # allgather_totals: all_gather_into_tensor on device (RCCL)
    assert gathered.device.type == "cuda" and gathered.shape == (1, 4)
    h = out.to_host()
    o = oracle.decode_batch(buf, off, lens, fmt, bf)
    assert_same(h, o, f"rccl {kind}")
    assert gathered.cpu().tolist()[0] == [o["n_kv"], o["key_bytes_total"], o["val_bytes_total"], o["n_restarts"]]
    # the direct helper on a device tensor
    t = torch.arange(4, dtype=torch.int64, device="cuda")
    assert allgather_totals(t).cpu().tolist() == [[0, 1, 2, 3]]


def test_bench_concat_step_over_rccl(nccl_group):
    """bench.py's per-step offset concat (concat_step + pbl_offset_concat) on
    the nccl group: the rebase by the (zero) exclusive prefix of lower ranks
    leaves rank 0's bases equal to the oracle's."""
    import torch
    import bench
    from pebble_amd.batch import BlockBatch, decode, offset_concat
    buf, off, lens, _ = gen_row_blocks(33, 128, 32768, 16, 16, 100)
    out = decode(BlockBatch.from_host(buf, off, lens, "cuda"))
    gathered = torch.zeros(4, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    bench.concat_step(nccl_group, gathered, out.totals[:32].view(torch.int64),
                      lambda g: offset_concat(out, g, 0, st))
    torch.cuda.synchronize()
    h = out.to_host()
    assert_same(h, oracle.decode_batch(buf, off, lens, N.PBL_FMT_ROW), "bench concat over rccl")
    assert gathered.cpu().tolist() == [h["n_kv"], h["key_bytes_total"], h["val_bytes_total"], h["n_restarts"]]
