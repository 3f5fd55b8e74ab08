"""Multi-rank sharding + offset concat over gloo.

CPU (world_size 2 and 4): each rank cuts its shard with the product's
partition_blocks + shard_host (the host half of ShardedBatchDecoder), decodes
it with the oracle (the device decode is covered by the gpu tests),
all-gathers its totals through allgather_totals, rebases its per-block bases
with exclusive_bases; the concatenation over ranks must equal a
single-process decode of the whole batch.  Mixed row + colblk batches
(config 4) slice the per-block formats alongside.

GPU (world_size 2, both ranks on cuda:0, gloo for the exchange): the product
ShardedBatchDecoder end to end, its device offset concat included.
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from pebble_amd import _native as N
from pebble_amd.colblk import gen_col_blocks
from pebble_amd.rowblk import gen_row_blocks
from pebble_amd.shard import allgather_totals, exclusive_bases, partition_blocks, shard_host

BASES = ["blk_kv_base", "blk_key_base", "blk_val_base", "blk_rst_base"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_batch(kind):
    """Row (config 2 shape) or mixed row + crdb1 colblk (config 4 shape, even
    ids row, odd ids colblk), small."""
    if kind == "row":
        buf, off, lens, _ = gen_row_blocks(77, 37, 8192, 16, 16, 100)
        return buf, off, lens, None
    rb, ro, rl, _ = gen_row_blocks(78, 12, 32768, 16, 16, 100)
    cb, co, cl, _ = gen_col_blocks(79, 11)
    nb = 23
    buf = np.zeros(nb * 32768 + 16, np.uint8)
    off = np.arange(nb, dtype=np.uint64) * 32768
    lens = np.zeros(nb, np.uint32)
    fmt = np.zeros(nb, np.uint8)
    for i in range(nb):
        src, so, sl, f = (rb, ro, rl, N.PBL_FMT_ROW) if i % 2 == 0 else (cb, co, cl, N.PBL_FMT_COL_CRDB1)
        k = i // 2
        buf[i * 32768: i * 32768 + int(sl[k])] = src[int(so[k]): int(so[k]) + int(sl[k])]
        lens[i], fmt[i] = sl[k], f
    return buf, off, lens, fmt


def _cpu_worker(rank, world, port, kind, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        buf, off, lens, fmt = make_batch(kind)
        s, e = partition_blocks(lens, world)[rank]
        sb, so, sl, sf = shard_host(buf, off, lens, s, e, fmt)
        o = oracle.decode_batch(sb, so, sl, 0, sf) if e > s else None
        local = torch.tensor([o["n_kv"], o["key_bytes_total"], o["val_bytes_total"], o["n_restarts"]]
                             if o else [0, 0, 0, 0], dtype=torch.int64)
        allt = allgather_totals(local)
        base = exclusive_bases(allt, rank).numpy().astype(np.uint64)
        res = {}
        if o:
            res = {k: (o[k][:-1] + base[i]) for i, k in enumerate(BASES)}
            res["keys"] = o["key_bytes"].tobytes()
            res["vals"] = o["val_bytes"].tobytes()
        q.put((rank, res, allt.numpy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, res, allt = q.get(timeout=300)
        results[r] = (res, allt)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


def _check_concat(results, world, kind):
    buf, off, lens, fmt = make_batch(kind)
    whole = oracle.decode_batch(buf, off, lens, 0, fmt)
    for k in BASES:
        cat = np.concatenate([results[r][0][k] for r in range(world) if results[r][0]])
        assert np.array_equal(cat, whole[k][:-1]), k
    assert b"".join(results[r][0]["keys"] for r in range(world) if results[r][0]) == whole["key_bytes"].tobytes()
    assert b"".join(results[r][0]["vals"] for r in range(world) if results[r][0]) == whole["val_bytes"].tobytes()
    # every rank saw the same gathered totals, summing to the batch totals
    allt = results[0][1]
    assert all(np.array_equal(results[r][1], allt) for r in range(world))
    assert allt[:, 0].sum() == whole["n_kv"]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("kind", ["row", "mixed"])
def test_sharded_offset_concat_gloo(world, kind):
    _check_concat(_run(_cpu_worker, world, kind), world, kind)


def _gpu_worker(rank, world, port, kind, q):
    import os
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from pebble_amd.shard import ShardedBatchDecoder
        torch.cuda.set_device(0)
        buf, off, lens, fmt = make_batch(kind)
        dec = ShardedBatchDecoder(buf, off, lens, N.PBL_FMT_ROW, 0, device="cuda:0", block_format=fmt)
        out, gathered = dec.decode()
        h = out.to_host()
        res = {k: h[k][:-1] for k in BASES}
        res["keys"] = h["key_bytes"].tobytes()
        res["vals"] = h["val_bytes"].tobytes()
        q.put((rank, res, gathered.cpu().numpy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["row", "mixed"])
def test_sharded_batch_decoder_two_ranks_gpu(kind):
    _check_concat(_run(_gpu_worker, 2, kind), 2, kind)


def test_partition_balances_bytes():
    lens = np.array([100] * 10 + [10000] + [100] * 10, np.uint32)
    parts = partition_blocks(lens, 4)
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    assert partition_blocks(lens, 1) == [(0, len(lens))]
    parts = partition_blocks(np.ones(1000, np.uint32), 8)
    sizes = [e - s for s, e in parts]
    assert max(sizes) - min(sizes) <= 1


def test_shard_host_keeps_phase_and_formats():
    buf = np.arange(200, dtype=np.uint8)
    off = np.array([3, 40, 77, 130], np.uint64)
    lens = np.array([30, 30, 40, 50], np.uint32)
    fmt = np.array([0, 2, 0, 1], np.uint8)
    sb, so, sl, sf = shard_host(buf, off, lens, 1, 3, fmt)
    assert list(sl) == [30, 40] and list(sf) == [2, 0]
    assert int(so[0]) % 16 == 40 % 16
    assert bytes(sb[int(so[0]): int(so[0]) + 30]) == bytes(buf[40:70])
    assert bytes(sb[int(so[1]): int(so[1]) + 40]) == bytes(buf[77:117])
    e = shard_host(buf, off, lens, 2, 2, fmt)
    assert len(e[1]) == 0 and len(e[3]) == 0
