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

from typing import List, Optional, Tuple

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
    """All-gather the 4 local totals (int64) of every rank -> [world, 4]."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty(world * 4, dtype=torch.int64, device=local_totals.device)
    if hasattr(dist, "all_gather_into_tensor") and local_totals.device.type == "cuda":
        dist.all_gather_into_tensor(out, local_totals.reshape(4).contiguous(), group=group)
    else:
        parts = [torch.empty(4, dtype=torch.int64, device=local_totals.device) for _ in range(world)]
        dist.all_gather(parts, local_totals.reshape(4).contiguous(), group=group)
        out = torch.cat(parts)
    return out.view(world, 4)


class ShardedBatchDecoder:
    """Decode this rank's shard of a host batch on its GPU and concat offsets.

    `decode()` returns the rank-local DecodedBatch whose blk_*_base arrays hold
    GLOBAL positions (as if the whole batch had been decoded on one device).
    """

    def __init__(self, blocks: np.ndarray, block_off: np.ndarray, block_len: np.ndarray, fmt: int = 0,
                 flags: int = 0, rank: Optional[int] = None, world: Optional[int] = None, device=None):
        import torch.distributed as dist
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        s, e = partition_blocks(block_len, self.world)[self.rank]
        self.block_range = (s, e)
        from .batch import BlockBatch
        if e > s:
            lo = int(block_off[s])
            hi = int(block_off[e - 1]) + int(block_len[e - 1])
            self.batch = BlockBatch.from_host(blocks[lo:hi], block_off[s:e] - lo, block_len[s:e], self.device,
                                              fmt, flags)
        else:
            self.batch = BlockBatch.from_host(np.zeros(16, np.uint8), np.zeros(0, np.uint64),
                                              np.zeros(0, np.uint32), self.device, fmt, flags)

    def decode(self, group=None):
        from .batch import decode, offset_concat
        out = decode(self.batch)
        local = out.totals[:32].view(torch.int64).clone()
        gathered = allgather_totals(local, group)
        offset_concat(out, gathered.reshape(-1).contiguous(), self.rank)
        torch.cuda.current_stream().synchronize()
        return out, gathered
