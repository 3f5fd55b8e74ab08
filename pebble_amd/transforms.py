"""blockiter.Transforms over a decoded batch on the device.

`apply_transforms(decoded, t)` runs `pbl_transform_batch` (pebble_amd/csrc/
transforms.hip): SyntheticSeqNum, HideObsoletePoints, SyntheticPrefix and
SyntheticSuffix (sstable/blockiter/transforms.go:20-248) applied to every block
of a batch `pbl_decode_batch` produced, into a new DecodedBatch with the same
layout contract.  Pebble applies them per KV inside rowblk.Iter / colblk.
DataBlockIter (rowblk_iter.go:400,487-517,1168-1187; data_block.go:1299-1303,
1437-1462,1680-1697); here it is one HBM-bound pass per batch.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _native as N
from .batch import BlockBatch, Capacity, DecodedBatch, DecodeError, _stream_handle
from .rowblk import Transforms

__all__ = ["Transforms", "TransformPlan", "apply_transforms"]


def _dev_bytes(b: bytes, device) -> Optional[torch.Tensor]:
    """Device copy of b, readable 16 bytes past its end (pbl_transform_batch
    copies by 16-B chunks)."""
    if not b:
        return None
    return torch.tensor(list(b) + [0] * 16, dtype=torch.uint8, device=device)


class TransformPlan:
    """Output buffers and ABI arguments of one transform of decoded batch `d`,
    built once and launched any number of times (`launch`): the bench's
    repeated transform pass, and `apply_transforms`."""

    def __init__(self, d: DecodedBatch, t: Transforms, stream=None, cap: Optional[Capacity] = None,
                 source: Optional[BlockBatch] = None):
        src = source if source is not None else d.source
        if src is None:
            raise DecodeError("apply_transforms needs the BlockBatch the decoded batch came from")
        tot = d.read_totals()
        n_kv, kb, vb, nr = int(tot.n_kv), int(tot.key_bytes), int(tot.val_bytes), int(tot.n_restarts)
        grow = len(t.synthetic_prefix) + len(t.synthetic_suffix)
        cap = cap or Capacity(kv=n_kv, key=kb + grow * n_kv, val=vb, rst=nr)
        dev = d.trailer.device
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        with torch.cuda.stream(st):
            out = DecodedBatch.allocate(d.n_blocks, cap, dev, entry_off=d.entry_off is not None,
                                        restarts=d.restarts is not None, meta=d.tiering_span_id is not None)
            ws = int(N.lib().pbl_transform_workspace_bytes(d.n_blocks))
            if out.workspace.numel() < ws:
                out.workspace = torch.empty(ws, dtype=torch.uint8, device=dev)
            self.pfx = _dev_bytes(t.synthetic_prefix, dev)
            self.sfx = _dev_bytes(t.synthetic_suffix, dev)
        self.d, self.out, self.stream = d, out, st
        self.sc = src.c_struct()
        self.tc = N.TransformsC(t.synthetic_seq_num, 1 if t.hide_obsolete_points else 0, t.split,
                                self.pfx.data_ptr() if self.pfx is not None else None,
                                self.sfx.data_ptr() if self.sfx is not None else None,
                                len(t.synthetic_prefix), len(t.synthetic_suffix), ctypes.pointer(self.sc))
        self.ic, self.oc = d.c_struct(), out.c_struct()

    def launch(self, stream=None) -> None:
        """pbl_transform_batch on `stream` (asynchronous)."""
        st = stream if stream is not None else self.stream
        rc = N.lib().pbl_transform_batch(ctypes.byref(self.ic), self.d.n_blocks, ctypes.byref(self.tc),
                                         ctypes.byref(self.oc), _stream_handle(st))
        if rc != N.PBL_OK:
            raise DecodeError(f"pbl_transform_batch failed: {N.STATUS_NAMES.get(rc, rc)}")


def apply_transforms(d: DecodedBatch, t: Transforms, stream=None, cap: Optional[Capacity] = None,
                     source: Optional[BlockBatch] = None) -> DecodedBatch:
    """Transform decoded batch `d` (its totals must be final: call after the
    decode's stream synchronised).  `source` is the BlockBatch `d` was decoded
    from (default `d.source`, which `decode()` records): row blocks are re-read
    where the synthetic prefix turns a key shorter than 8 B into a valid one
    (rowblk_iter.go:400,1168-1199).  Output capacities default to exact upper
    bounds: every KV kept, every key grown by prefix + suffix (a key made valid
    by the prefix has a user key inside the prefix, so the bound holds)."""
    plan = TransformPlan(d, t, stream, cap, source)
    plan.launch()
    plan.stream.synchronize()
    plan.out.read_totals()
    return plan.out
