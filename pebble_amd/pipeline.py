"""Host-resident blocks through the device and back: the PCIe-inclusive path.

A Go caller's blocks arrive in host memory (the block cache / a file read);
this streams them through H2D -> `pbl_decode_batch` -> D2H of the decoded
arrays, full duplex:

  h2d stream     chunk c's blocks, lengths and (rebased) offsets in
  decode stream  waits for c's H2D and for its slot's previous D2H, decodes c,
                 copies c's 64-B totals to pinned memory
  d2h stream     c's decoded arrays out, EXACT sizes

Three HIP streams (GPU_MAX_HW_QUEUES is 4 on the box: each gets its own
hardware queue), `slots` device buffer sets (default 3) so that chunk c+1's
H2D, chunk c's decode and chunk c-1's D2H run at the same time.  The host
blocks only on a chunk's totals event, and only after it has queued the H2D
and decode of the next `slots - 1` chunks: the GPU always has queued work.
The D2H of a chunk is queued as soon as its totals are known (they size the
copies), so no bytes beyond the decoded ones cross PCIe.

Decoded arrays land in one pinned host region per array, chunk after chunk;
`ChunkResult` carries each chunk's totals and where its bytes start (the
offsets inside a chunk are chunk-relative, as `pbl_decode_batch` writes them).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _native as N
from .batch import BlockBatch, Capacity, DecodedBatch, DecodeError, decode_into, varlen_hint

# arrays brought back per chunk: (DecodedBatch field, bytes per unit, unit)
D2H_ARRAYS = (("trailer", 8, "kv"), ("kv_flags", 1, "kv"), ("key_off", 4, "kvb"), ("val_off", 4, "kvb"),
              ("key_bytes", 1, "key"), ("val_bytes", 1, "val"))


@dataclass
class ChunkResult:
    first_block: int
    n_blocks: int
    n_kv: int
    key_bytes: int
    val_bytes: int
    status_mask: int
    host_pos: dict  # array name -> byte offset of this chunk's data in HostOutputs


@dataclass
class HostOutputs:
    arrays: dict  # name -> pinned uint8 torch tensor
    chunks: List[ChunkResult]

    def view(self, c: int, name: str, dtype) -> np.ndarray:
        ch = self.chunks[c]
        n = {"trailer": ch.n_kv * 8, "kv_flags": ch.n_kv, "key_off": 4 * (ch.n_kv + ch.n_blocks),
             "val_off": 4 * (ch.n_kv + ch.n_blocks), "key_bytes": ch.key_bytes, "val_bytes": ch.val_bytes}[name]
        p = ch.host_pos[name]
        return self.arrays[name][p:p + n].numpy().view(dtype)


class HostPipeline:
    """Reusable device state for streaming host batches (one device)."""

    def __init__(self, device, chunk_blocks: int, chunk_bytes: int, per_chunk: Capacity, slots: int = 3):
        self.dev = torch.device(device)
        self.chunk_blocks = chunk_blocks
        self.slots = slots
        self.per = per_chunk
        self.h2d = torch.cuda.Stream(self.dev)
        self.dec = torch.cuda.Stream(self.dev)
        self.d2h = torch.cuda.Stream(self.dev)
        self.s = []
        for _ in range(slots):
            self.s.append({
                "blocks": torch.empty(chunk_bytes + 16, dtype=torch.uint8, device=self.dev),
                "off": torch.empty(chunk_blocks, dtype=torch.int64, device=self.dev),
                "len": torch.empty(chunk_blocks, dtype=torch.int32, device=self.dev),
                "fmt": torch.empty(chunk_blocks, dtype=torch.uint8, device=self.dev),
                "out": DecodedBatch.allocate(chunk_blocks, per_chunk, self.dev, entry_off=False, restarts=False),
                "tot": torch.empty(ctypes_sizeof_totals(), dtype=torch.uint8).pin_memory(),
                "ev_in": torch.cuda.Event(), "ev_dec": torch.cuda.Event(), "ev_out": torch.cuda.Event(),
                "used": False,
            })

    def run(self, host_blocks: torch.Tensor, off: np.ndarray, lens: np.ndarray, fmt: int, flags: int,
            out: HostOutputs, block_format: Optional[np.ndarray] = None) -> HostOutputs:
        """Stream every block of a pinned host batch; fills `out` (pinned)."""
        assert host_blocks.is_pinned()
        nb = len(off)
        cb = self.chunk_blocks
        nch = (nb + cb - 1) // cb
        off = np.ascontiguousarray(off, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        # per-chunk rebased offsets and lengths, pinned (the index a caller holds)
        h_off = torch.empty(nb, dtype=torch.int64).pin_memory()
        h_len = torch.from_numpy(lens.view(np.int32)).pin_memory()
        h_fmt = None if block_format is None else torch.from_numpy(np.ascontiguousarray(block_format, np.uint8)).pin_memory()
        starts = []
        for c in range(nch):
            b0, b1 = c * cb, min(nb, (c + 1) * cb)
            lo = int(off[b0])
            hi = int((off[b0:b1] + lens[b0:b1]).max())
            if hi - lo + 16 > self.s[0]["blocks"].numel():
                raise ValueError("chunk larger than the pipeline's chunk_bytes")
            h_off[b0:b1] = torch.from_numpy((off[b0:b1] - np.uint64(lo)).view(np.int64))
            starts.append((b0, b1, lo, hi))
        hpos = {name: 0 for name, _, _ in D2H_ARRAYS}
        out.chunks.clear()

        def queue_in(c):
            b0, b1, lo, hi = starts[c]
            S = self.s[c % self.slots]
            with torch.cuda.stream(self.h2d):
                if S["used"]:
                    self.h2d.wait_event(S["ev_dec"])  # the slot's previous chunk has been decoded
                n = b1 - b0
                S["blocks"][: hi - lo].copy_(host_blocks[lo:hi], non_blocking=True)
                S["off"][:n].copy_(h_off[b0:b1], non_blocking=True)
                S["len"][:n].copy_(h_len[b0:b1], non_blocking=True)
                if h_fmt is not None:
                    S["fmt"][:n].copy_(h_fmt[b0:b1], non_blocking=True)
                S["ev_in"].record(self.h2d)
            with torch.cuda.stream(self.dec):
                self.dec.wait_event(S["ev_in"])
                if S["used"]:
                    self.dec.wait_event(S["ev_out"])  # the slot's previous outputs have left
                bb = BlockBatch(S["blocks"], S["off"][:n], S["len"][:n], fmt, flags | varlen_hint(lens[b0:b1]),
                                S["fmt"][:n] if h_fmt is not None else None)
                decode_into(bb, S["out"], self.dec)
                S["tot"].copy_(S["out"].totals, non_blocking=True)
                S["ev_dec"].record(self.dec)
            S["used"] = True

        def queue_out(c):
            b0, b1, _, _ = starts[c]
            S = self.s[c % self.slots]
            S["ev_dec"].synchronize()  # this chunk's totals (the next chunks are already queued)
            t = N.TotalsC.from_buffer_copy(S["tot"].numpy().tobytes())
            n = b1 - b0
            if t.status_mask & (1 << N.PBL_OVERFLOW):
                raise DecodeError(f"chunk {c}: per-chunk capacity exceeded")
            units = {"kv": int(t.n_kv), "kvb": int(t.n_kv) + n, "key": int(t.key_bytes), "val": int(t.val_bytes)}
            o = S["out"]
            pos = {}
            with torch.cuda.stream(self.d2h):
                for name, w, u in D2H_ARRAYS:
                    nbytes = w * units[u]
                    dst = out.arrays[name]
                    if hpos[name] + nbytes > dst.numel():
                        raise DecodeError(f"host output {name} too small")
                    src = getattr(o, name).view(torch.uint8)[:nbytes]
                    if nbytes:
                        dst[hpos[name]:hpos[name] + nbytes].copy_(src, non_blocking=True)
                    pos[name] = hpos[name]
                    hpos[name] += nbytes
                S["ev_out"].record(self.d2h)
            out.chunks.append(ChunkResult(b0, n, int(t.n_kv), int(t.key_bytes), int(t.val_bytes), int(t.status_mask),
                                          pos))

        ahead = self.slots - 1
        for c in range(min(ahead, nch)):
            queue_in(c)
        for c in range(nch):
            if c + ahead < nch:
                queue_in(c + ahead)
            queue_out(c)
        self.d2h.synchronize()
        return out


def ctypes_sizeof_totals() -> int:
    import ctypes
    return ctypes.sizeof(N.TotalsC)


def host_outputs(cap: Capacity, n_blocks: int) -> HostOutputs:
    """Pinned host arrays large enough for a whole batch of `cap` totals."""
    sizes = {"trailer": 8 * cap.kv, "kv_flags": cap.kv, "key_off": 4 * (cap.kv + n_blocks),
             "val_off": 4 * (cap.kv + n_blocks), "key_bytes": cap.key, "val_bytes": cap.val}
    return HostOutputs({k: torch.empty(max(v, 1), dtype=torch.uint8).pin_memory() for k, v in sizes.items()}, [])


def stream_batch(host_blocks: torch.Tensor, off, lens, fmt: int, flags: int, cap: Capacity, device,
                 chunk_blocks: int = 4096, slots: int = 3, block_format=None, pipe: Optional[HostPipeline] = None,
                 outputs: Optional[HostOutputs] = None):
    """One pass of a pinned host batch through a (new or given) pipeline.
    Returns (HostOutputs, seconds, pipeline)."""
    nb = len(off)
    if pipe is None:
        off = np.asarray(off, np.uint64)
        lens = np.asarray(lens, np.uint32)
        span = 0
        for b0 in range(0, nb, chunk_blocks):
            b1 = min(nb, b0 + chunk_blocks)
            span = max(span, int((off[b0:b1] + lens[b0:b1]).max() - off[b0]))
        frac = min(1.0, chunk_blocks / max(nb, 1))
        per = Capacity(kv=int(cap.kv * frac * 1.5) + 4096, key=int(cap.key * frac * 1.5) + 65536,
                       val=int(cap.val * frac * 1.5) + 65536, rst=0)
        pipe = HostPipeline(device, chunk_blocks, span, per, slots)
    outputs = outputs or host_outputs(cap, nb)
    torch.cuda.synchronize(pipe.dev)
    t0 = time.perf_counter()
    pipe.run(host_blocks, off, lens, fmt, flags, outputs, block_format)
    return outputs, time.perf_counter() - t0, pipe
