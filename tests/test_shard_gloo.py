"""Multi-rank sharding + offset concat on CPU (gloo, world_size 2 and 4).

Each rank decodes its contiguous shard with the oracle (the device decode is
covered by the gpu tests), all-gathers its totals through
pebble_amd.shard.allgather_totals, rebases its per-block bases with
exclusive_bases, and the concatenation of every rank's rebased bases must
equal a single-process decode of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from pebble_amd.rowblk import gen_row_blocks
from pebble_amd.shard import allgather_totals, exclusive_bases, partition_blocks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        buf, off, lens, n = gen_row_blocks(77, 37, 8192, 16, 16, 100)
        # ragged sizes: drop some KVs from a few blocks by truncating their length field
        s, e = partition_blocks(lens, world)[rank]
        o = oracle.rowblk_decode_batch(buf, off[s:e], lens[s:e]) if e > s else None
        local = torch.tensor([o["n_kv"], o["key_bytes_total"], o["val_bytes_total"], o["n_restarts"]]
                             if o else [0, 0, 0, 0], dtype=torch.int64)
        allt = allgather_totals(local)
        base = exclusive_bases(allt, rank).numpy().astype(np.uint64)
        res = {}
        if o:
            res = {k: (o[k][:-1] + base[i]) for i, k in enumerate(["blk_kv_base", "blk_key_base", "blk_val_base",
                                                                     "blk_rst_base"])}
            res["range"] = (s, e)
            res["keys"] = o["key_bytes"].tobytes()
        q.put((rank, res, allt.numpy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_offset_concat_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict()
    for _ in range(world):
        r, res, allt = q.get(timeout=120)
        results[r] = (res, allt)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, off, lens, n = gen_row_blocks(77, 37, 8192, 16, 16, 100)
    whole = oracle.rowblk_decode_batch(buf, off, lens)
    for k in ["blk_kv_base", "blk_key_base", "blk_val_base", "blk_rst_base"]:
        cat = np.concatenate([results[r][0][k] for r in range(world) if results[r][0]])
        assert np.array_equal(cat, whole[k][:-1]), k
    keys = b"".join(results[r][0]["keys"] for r in range(world) if results[r][0])
    assert keys == whole["key_bytes"].tobytes()
    # every rank saw the same gathered totals, summing to the batch totals
    allt = results[0][1]
    assert all(np.array_equal(results[r][1], allt) for r in range(world))
    assert allt[:, 0].sum() == whole["n_kv"]


def test_partition_balances_bytes():
    lens = np.array([100] * 10 + [10000] + [100] * 10, np.uint32)
    parts = partition_blocks(lens, 4)
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    assert partition_blocks(lens, 1) == [(0, len(lens))]
    parts = partition_blocks(np.ones(1000, np.uint32), 8)
    sizes = [e - s for s, e in parts]
    assert max(sizes) - min(sizes) <= 1
