"""Multi-GPU sharding of a block batch.

Blocks are independent, so a batch is split into contiguous block ranges of
~equal input bytes, one per rank (one process per GPU).  Each rank decodes its
range with no data-path collective; the only exchange is the *offset concat*:
an all-gather of every rank's 4 totals {n_kv, key_bytes, val_bytes,
n_restarts} (RCCL over xGMI on GPUs, gloo on CPU), after which each rank adds
the exclusive prefix of the lower ranks to its per-block bases.  Per-KV
offsets are block-relative and never move; decoded bytes stay on their GPU.
"""
from __future__ import annotations

from typing import List, Optional, Tuple  # noqa: F401

import numpy as np
import torch


def partition_blocks(block_len: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) block ranges per rank, balanced by input bytes
    (config 5's variable block sizes make count-balancing uneven)."""
    n = len(block_len)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    csum = np.concatenate([[0], np.cumsum(block_len.astype(np.int64))])
    total = int(csum[-1])
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        i = int(np.searchsorted(csum, target, side="left"))
        i = min(max(i, bounds[-1]), n)
        bounds.append(i)
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def exclusive_bases(all_totals: torch.Tensor, rank: int) -> torch.Tensor:
    """Exclusive prefix over lower ranks of the all-gathered [world, 4] totals."""
    t = all_totals.view(-1, 4).to(torch.int64)
    if rank == 0:
        return torch.zeros(4, dtype=torch.int64, device=t.device)
    return t[:rank].sum(0)


def allgather_totals(local_totals: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather the 4 local totals (int64) of every rank -> [world, 4], on the
    device of `local_totals`.  RCCL (backend "nccl") gathers device tensors in
    place; a gloo group gathers through host memory."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = local_totals.device
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * 4, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, local_totals.reshape(4).contiguous(), group=group)
        return out.view(world, 4)
    loc = local_totals.reshape(4).to("cpu", torch.int64).contiguous()
    parts = [torch.empty(4, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, loc, group=group)
    return torch.cat(parts).to(dev).view(world, 4)


def shard_host(blocks: np.ndarray, block_off: np.ndarray, block_len: np.ndarray, start: int, end: int,
               block_format: Optional[np.ndarray] = None):
    """The host bytes and descriptors of blocks [start, end): (buf, off, lens,
    block_format) with offsets relative to the shard's first byte (its 16-B
    phase kept, so the device sees every block at the same alignment)."""
    if end <= start:
        return (np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                None if block_format is None else np.zeros(0, np.uint8))
    lo = int(block_off[start]) & ~15
    hi = int((block_off[start:end].astype(np.int64) + block_len[start:end].astype(np.int64)).max())
    buf = np.ascontiguousarray(blocks[lo:hi])
    off = (block_off[start:end].astype(np.uint64) - np.uint64(lo)).astype(np.uint64)
    lens = np.ascontiguousarray(block_len[start:end], dtype=np.uint32)
    bf = None if block_format is None else np.ascontiguousarray(block_format[start:end], dtype=np.uint8)
    return buf, off, lens, bf


class ShardedBatchDecoder:
    """Decode this rank's shard of a host batch on its GPU and concat offsets
    (SURVEY.md §8(e)).

    Rank r takes the contiguous block range `partition_blocks(block_len,
    world)[r]` (formats sliced alongside for mixed batches, config 4).
    `decode()` returns the rank-local DecodedBatch whose blk_*_base arrays hold
    GLOBAL positions (as if the whole batch had been decoded on one device),
    and the gathered [world, 4] totals.
    """

    def __init__(self, blocks: np.ndarray, block_off: np.ndarray, block_len: np.ndarray, fmt: int = 0,
                 flags: int = 0, rank: Optional[int] = None, world: Optional[int] = None, device=None,
                 block_format: Optional[np.ndarray] = None):
        import torch.distributed as dist
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        s, e = partition_blocks(block_len, self.world)[self.rank]
        self.block_range = (s, e)
        from .batch import BlockBatch
        buf, off, lens, bf = shard_host(blocks, block_off, block_len, s, e, block_format)
        self.batch = BlockBatch.from_host(buf, off, lens, self.device, fmt, flags, block_format=bf)

    def decode(self, group=None, gather=allgather_totals):
        """Decode the shard, exchange totals (`gather`: the all-gather, or a
        stand-in returning the [world, 4] totals for single-process tests) and
        rebase this rank's per-block bases on device."""
        from .batch import decode, offset_concat
        out = decode(self.batch)
        local = out.totals[:32].view(torch.int64).clone()
        gathered = gather(local, group)
        offset_concat(out, gathered.reshape(-1).contiguous(), self.rank)
        torch.cuda.current_stream(self.device).synchronize()
        return out, gathered
