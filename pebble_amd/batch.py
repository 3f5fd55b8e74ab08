"""Device-resident block batches and the batch decode (host side of the C-ABI).

A `BlockBatch` holds raw, already-decompressed data blocks in HBM; `decode()`
runs the single-pass HIP decoder over it and returns a `DecodedBatch` whose
arrays follow include/pebble_amd.h exactly.  torch is only plumbing here
(device memory, streams); the work is done by libpebble_amd.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _native as N


def _dp(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class DecodeError(RuntimeError):
    pass


def _row_entries(blk: bytes) -> int:
    """Entries of one row block by its header chain (rowblk_iter.go:345-398;
    -1 if the block does not parse): the sampling behind varlen_hint."""
    n = len(blk)
    if n < 4:
        return -1
    nres = int.from_bytes(blk[n - 4:], "little")
    roff = n - 4 * (1 + nres)
    if nres == 0 or roff < 0:
        return -1
    off, k = 0, 0
    while off < roff:
        vals = []
        for _ in range(3):
            v, sh = 0, 0
            while True:
                if off >= n or sh > 28:
                    return -1
                c = blk[off]
                off += 1
                v |= (c & 0x7F) << sh
                sh += 7
                if c < 0x80:
                    break
            vals.append(v)
        off += vals[1] + vals[2]
        k += 1
    return k


def varlen_hint(lens: np.ndarray, blocks: Optional[np.ndarray] = None, off: Optional[np.ndarray] = None,
                fmt: int = N.PBL_FMT_ROW, sample: int = 16) -> int:
    """PBL_BATCH_VARLEN when block lengths vary widely (coefficient of variation
    above 0.25): a scheduling hint only (include/pebble_amd.h).  With the
    host bytes of a row batch, also only when its blocks are value-dominated:
    `sample` evenly spaced blocks average at most 64 entries (config 5: ~13).
    Row blocks of many small KVs (config 2's 271) decode faster on the pool
    kernel even when their lengths vary (a row-shape mix of config-2 blocks
    and short tails: 940 GiB/s in the two-pass form against 1227)."""
    l = np.asarray(lens, dtype=np.float64)
    if l.size < 2 or l.mean() <= 0 or l.std() / l.mean() <= 0.25:
        return 0
    if blocks is not None and off is not None and fmt == N.PBL_FMT_ROW:
        idx = np.unique(np.linspace(0, l.size - 1, min(sample, l.size)).astype(np.int64))
        counts = [_row_entries(bytes(blocks[int(off[i]): int(off[i]) + int(lens[i])])) for i in idx]
        counts = [c for c in counts if c >= 0]
        if counts and sum(counts) / len(counts) > 64:
            return 0
    return N.PBL_BATCH_VARLEN


@dataclass
class BlockBatch:
    """Raw data blocks resident on one device (concatenated, 16-B readable slack)."""
    blocks: torch.Tensor        # uint8 [bytes (+16 pad)]
    block_off: torch.Tensor     # int64 [n]  (uint64 in the ABI)
    block_len: torch.Tensor     # int32 [n]  (uint32 in the ABI)
    format: int = N.PBL_FMT_ROW
    flags: int = 0
    block_format: Optional[torch.Tensor] = None  # uint8 [n] per-block PBL_FMT_* (mixed batches)
    synthetic_seq_num: int = 0  # blockiter.SyntheticSeqNum fused into the decode (0 = unset)

    @property
    def n_blocks(self) -> int:
        return int(self.block_off.numel())

    @property
    def device(self) -> torch.device:
        return self.blocks.device

    @classmethod
    def from_host(cls, blocks: np.ndarray, off: np.ndarray, lens: np.ndarray, device="cuda",
                  fmt: int = N.PBL_FMT_ROW, flags: int = 0, non_blocking: bool = False,
                  block_format: Optional[np.ndarray] = None) -> "BlockBatch":
        blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
        pad = np.zeros(len(blocks) + 16, np.uint8)
        pad[: len(blocks)] = blocks
        b = torch.from_numpy(pad).to(device, non_blocking=non_blocking)
        o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).to(device)
        l = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint32).view(np.int32)).to(device)
        flags |= varlen_hint(lens, blocks, off, fmt if block_format is None else -1)
        bf = None
        if block_format is not None:
            bf = torch.from_numpy(np.ascontiguousarray(block_format, dtype=np.uint8)).to(device)
        return cls(b, o, l, fmt, flags, bf)

    @classmethod
    def from_blocks(cls, blocks: list, device="cuda", fmt: int = N.PBL_FMT_ROW, flags: int = 0,
                    align: int = 8, block_format=None) -> "BlockBatch":
        """Pack a list of block byte strings (each start `align`-aligned)."""
        offs, lens, pos = [], [], 0
        for bk in blocks:
            pos = (pos + align - 1) // align * align
            offs.append(pos)
            lens.append(len(bk))
            pos += len(bk)
        buf = np.zeros(max(pos, 1), np.uint8)
        for o, bk in zip(offs, blocks):
            buf[o:o + len(bk)] = np.frombuffer(bk, np.uint8)
        return cls.from_host(buf, np.array(offs, np.uint64), np.array(lens, np.uint32), device, fmt, flags,
                             block_format=None if block_format is None else np.asarray(block_format, np.uint8))

    def c_struct(self) -> N.BlockBatchC:
        return N.BlockBatchC(self.blocks.data_ptr(), self.block_off.data_ptr(), self.block_len.data_ptr(),
                             self.n_blocks, self.format, self.flags, 0,
                             self.block_format.data_ptr() if self.block_format is not None else None,
                             self.synthetic_seq_num)

    def input_bytes(self) -> int:
        return int(self.block_len.to(torch.int64).sum().item()) if self.n_blocks else 0


@dataclass
class Capacity:
    kv: int
    key: int
    val: int
    rst: int

    @classmethod
    def estimate(cls, batch: BlockBatch) -> "Capacity":
        tot = max(batch.input_bytes(), 1)
        nb = batch.n_blocks
        # values never exceed the input; keys and KV counts are heuristics that
        # are corrected by one re-run when the kernel reports PBL_OVERFLOW.
        return cls(kv=tot // 24 + 64 * nb + 64, key=tot // 2 + 64, val=tot + 64, rst=tot // 16 + 16 * nb + 16)


@dataclass
class DecodedBatch:
    n_blocks: int
    trailer: torch.Tensor
    kv_flags: torch.Tensor
    entry_off: Optional[torch.Tensor]
    key_off: torch.Tensor
    val_off: torch.Tensor
    key_bytes: torch.Tensor
    val_bytes: torch.Tensor
    restarts: Optional[torch.Tensor]
    blk_kv_base: torch.Tensor
    blk_key_base: torch.Tensor
    blk_val_base: torch.Tensor
    blk_rst_base: torch.Tensor
    blk_status: torch.Tensor
    totals: torch.Tensor          # uint8 view of pbl_totals
    workspace: torch.Tensor
    cap: Capacity
    _host_totals: Optional[N.TotalsC] = field(default=None, repr=False)
    source: Optional[BlockBatch] = field(default=None, repr=False)  # the batch it was decoded from
    # base.KVMeta per KV (Pebblev8 tiering, PBL_COL_TIERING); None = not requested
    tiering_span_id: Optional[torch.Tensor] = None
    tiering_attr: Optional[torch.Tensor] = None

    @classmethod
    def allocate(cls, n_blocks: int, cap: Capacity, device, entry_off: bool = True,
                 restarts: bool = True, meta: bool = False) -> "DecodedBatch":
        d = torch.device(device)
        u = lambda n, dt: torch.empty(max(int(n), 1), dtype=dt, device=d)  # noqa: E731
        lib = N.lib()
        ws = int(lib.pbl_workspace_bytes(n_blocks))
        return cls(
            n_blocks=n_blocks,
            trailer=u(cap.kv, torch.int64), kv_flags=u(cap.kv, torch.uint8),
            entry_off=u(cap.kv, torch.int32) if entry_off else None,
            key_off=u(cap.kv + n_blocks, torch.int32), val_off=u(cap.kv + n_blocks, torch.int32),
            key_bytes=u(cap.key + 16, torch.uint8), val_bytes=u(cap.val + 16, torch.uint8),
            restarts=u(cap.rst, torch.int32) if restarts else None,
            blk_kv_base=u(n_blocks + 1, torch.int64), blk_key_base=u(n_blocks + 1, torch.int64),
            blk_val_base=u(n_blocks + 1, torch.int64), blk_rst_base=u(n_blocks + 1, torch.int64),
            blk_status=u(n_blocks, torch.int32),
            totals=torch.zeros(ctypes.sizeof(N.TotalsC), dtype=torch.uint8, device=d),
            workspace=u(ws, torch.uint8), cap=cap,
            tiering_span_id=u(cap.kv, torch.int64) if meta else None,
            tiering_attr=u(cap.kv, torch.int64) if meta else None,
        )

    def c_struct(self) -> N.DecodeOutC:
        c = self.cap
        return N.DecodeOutC(
            self.trailer.data_ptr(), self.kv_flags.data_ptr(),
            self.entry_off.data_ptr() if self.entry_off is not None else None,
            self.key_off.data_ptr(), self.val_off.data_ptr(), self.key_bytes.data_ptr(),
            self.val_bytes.data_ptr(), self.restarts.data_ptr() if self.restarts is not None else None,
            self.blk_kv_base.data_ptr(), self.blk_key_base.data_ptr(), self.blk_val_base.data_ptr(),
            self.blk_rst_base.data_ptr(), self.blk_status.data_ptr(), self.totals.data_ptr(),
            c.kv, c.key, c.val, c.rst if self.restarts is not None else 0,
            self.workspace.data_ptr(), self.workspace.numel(),
            _dp(self.tiering_span_id), _dp(self.tiering_attr),
        )

    # ---- host readouts ------------------------------------------------------------
    def read_totals(self) -> N.TotalsC:
        raw = self.totals.cpu().numpy().tobytes()  # (a sync copy: call after the decode's stream)
        t = N.TotalsC.from_buffer_copy(raw)
        self._host_totals = t
        return t

    def to_host(self) -> dict:
        """Copy every array back (sized by the totals) as numpy, oracle layout."""
        t = self.read_totals()
        nb, n = self.n_blocks, int(t.n_kv)
        g = lambda x, k, dt: x[:k].cpu().numpy().view(dt) if k else np.zeros(0, dt)  # noqa: E731
        r = {
            "trailer": g(self.trailer, n, np.uint64), "kv_flags": g(self.kv_flags, n, np.uint8),
            "entry_off": g(self.entry_off, n, np.uint32) if self.entry_off is not None else None,
            "key_off": g(self.key_off, n + nb, np.uint32), "val_off": g(self.val_off, n + nb, np.uint32),
            "key_bytes": g(self.key_bytes, int(t.key_bytes), np.uint8),
            "val_bytes": g(self.val_bytes, int(t.val_bytes), np.uint8),
            "restarts": g(self.restarts, int(t.n_restarts), np.uint32) if self.restarts is not None else None,
            "blk_kv_base": g(self.blk_kv_base, nb + 1, np.uint64),
            "blk_key_base": g(self.blk_key_base, nb + 1, np.uint64),
            "blk_val_base": g(self.blk_val_base, nb + 1, np.uint64),
            "blk_rst_base": g(self.blk_rst_base, nb + 1, np.uint64),
            "blk_status": g(self.blk_status, nb, np.uint32),
            "n_kv": n, "key_bytes_total": int(t.key_bytes), "val_bytes_total": int(t.val_bytes),
            "n_restarts": int(t.n_restarts), "status_mask": int(t.status_mask),
            "n_bad_blocks": int(t.n_bad_blocks), "n_slow_blocks": int(t.n_slow_blocks),
        }
        if self.tiering_span_id is not None:
            r["tiering_span_id"] = g(self.tiering_span_id, n, np.uint64)
            r["tiering_attr"] = g(self.tiering_attr, n, np.uint64)
        return r


def decode_into(batch: BlockBatch, out: DecodedBatch, stream=None) -> None:
    """Launch the decode of `batch` into preallocated `out` (asynchronous)."""
    lib = N.lib()
    b = batch.c_struct()
    o = out.c_struct()
    rc = lib.pbl_decode_batch(ctypes.byref(b), ctypes.byref(o), _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_decode_batch failed: {N.STATUS_NAMES.get(rc, rc)}")


def size_batch(batch: BlockBatch, stream=None) -> DecodedBatch:
    """Size pass (`pbl_size_batch`): per-block bases, statuses and totals only,
    in a DecodedBatch whose per-KV arrays are empty (Capacity 0)."""
    st = stream if stream is not None else torch.cuda.current_stream(batch.device)
    with torch.cuda.stream(st):
        out = DecodedBatch.allocate(batch.n_blocks, Capacity(0, 0, 0, 0), batch.device)
    b = batch.c_struct()
    o = out.c_struct()
    rc = N.lib().pbl_size_batch(ctypes.byref(b), ctypes.byref(o), ctypes.c_void_p(st.cuda_stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_size_batch failed: {N.STATUS_NAMES.get(rc, rc)}")
    return out


def decode(batch: BlockBatch, cap: Optional[Capacity] = None, stream=None, entry_off: bool = True,
           restarts: bool = True, exact: bool = False, meta: bool = False) -> DecodedBatch:
    """Decode a batch.  Without `cap`, capacities are estimated and the decode
    re-runs once with exact ones on PBL_OVERFLOW; `exact=True` runs the size
    pass first instead (one parse more, never a second decode).  The outputs are
    allocated on the launch stream, so the caching allocator never hands them to
    other work while the kernel writes them.  `meta`: also the per-KV KVMeta
    arrays (the tiering columns of PBL_COL_TIERING batches; zeros otherwise)."""
    st = stream if stream is not None else torch.cuda.current_stream(batch.device)
    if cap is None and exact:
        sz = size_batch(batch, st)
        st.synchronize()
        t = sz.read_totals()
        cap = Capacity(kv=int(t.n_kv), key=int(t.key_bytes), val=int(t.val_bytes), rst=int(t.n_restarts))
    cap = cap or Capacity.estimate(batch)
    with torch.cuda.stream(st):
        out = DecodedBatch.allocate(batch.n_blocks, cap, batch.device, entry_off, restarts, meta)
    decode_into(batch, out, st)
    out.source = batch
    st.synchronize()
    t = out.read_totals()
    if t.status_mask & (1 << N.PBL_OVERFLOW):
        cap = Capacity(kv=int(t.n_kv) + 1, key=int(t.key_bytes) + 1, val=int(t.val_bytes) + 1,
                       rst=int(t.n_restarts) + 1)
        with torch.cuda.stream(st):
            out = DecodedBatch.allocate(batch.n_blocks, cap, batch.device, entry_off, restarts, meta)
        decode_into(batch, out, st)
        out.source = batch
        st.synchronize()
        out.read_totals()
    return out


def rebase(out: DecodedBatch, kv: int, key: int, val: int, rst: int, stream=None) -> None:
    """Offset concat for a sharded batch: add this rank's global bases."""
    lib = N.lib()
    o = out.c_struct()
    rc = lib.pbl_rebase_blocks(ctypes.byref(o), out.n_blocks, kv, key, val, rst, _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_rebase_blocks failed: {N.STATUS_NAMES.get(rc, rc)}")


def offset_concat(out: DecodedBatch, rank_totals: torch.Tensor, rank: int, stream=None) -> None:
    """Device-side offset concat: `rank_totals` is the int64 [world*4] tensor an
    RCCL all-gather of every rank's totals prefix produced."""
    lib = N.lib()
    o = out.c_struct()
    rc = lib.pbl_offset_concat(ctypes.byref(o), out.n_blocks, ctypes.c_void_p(rank_totals.data_ptr()), rank,
                               _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_offset_concat failed: {N.STATUS_NAMES.get(rc, rc)}")


def gen_zipf_blocks(seed: int, n_blocks: int, fmt: int = 0, restart_interval: int = 16, block_size: int = 32768,
                    key_min: int = 8, key_max: int = 1024, val_min: int = 0, val_max: int = 65536, s: float = 1.1,
                    n_threads: int = 0, first_block: int = 0):
    """Config 5 (BASELINE.json configs[4]): Zipf(s) key lengths in [key_min, key_max]
    and value lengths in [val_min, val_max], variable-length blocks packed at 8-B
    alignment (`pbl_gen_zipf_blocks`).  fmt is PBL_FMT_ROW or PBL_FMT_COL_DEFAULT.
    Block i is global block first_block + i of the seed's batch (a rank's shard).
    Returns (buf, off, lens, n_kv) with buf padded by 16 zero bytes."""
    import ctypes
    import os
    cfg = N.ZipfConfigC(seed, key_min, key_max, val_min, val_max, s, block_size, restart_interval, first_block, 0)
    nt = n_threads or min(16, os.cpu_count() or 1)
    off = np.empty(n_blocks, np.uint64)
    lens = np.empty(n_blocks, np.uint32)
    used = ctypes.c_uint64(0)
    # worst case: every block is its target plus one maximal KV
    cap = n_blocks * (block_size + key_max + val_max + 64)
    buf = np.empty(cap + 16, np.uint8)
    n = N.gen_lib().pbl_gen_zipf_blocks(ctypes.byref(cfg), fmt, n_blocks, buf.ctypes.data, cap, off.ctypes.data,
                                    lens.ctypes.data, ctypes.byref(used), nt)
    if n == (1 << 64) - 1:
        raise ValueError(f"pbl_gen_zipf_blocks: bad config or capacity ({used.value} > {cap})")
    buf = buf[: used.value + 16].copy()
    buf[used.value:] = 0
    return buf, off, lens, int(n)


def gen_row_mix(seed: int, n_blocks: int, kind: str = "zipf10", n_threads: int = 0):
    """Row batches whose block shapes vary inside one batch (the shapes a
    compaction or a multi-table read hands over), for the per-block kernel
    routing: "zipf10" = config-2 blocks with every 10th block a config-5 Zipf
    block (restart interval 16); "tail8" = config-2 blocks with every 8th block
    a table's short last block (2, 4 or 8 KiB, the same 16 B / 100 B KVs).
    Blocks packed at 8-B aligned offsets.  Returns (buf, off, lens, n_kv)."""
    from .rowblk import gen_row_blocks
    ids = np.arange(n_blocks)
    if kind == "zipf10":
        odd = ids % 10 == 9
        a_buf, a_off, a_len, a_n = gen_row_blocks(seed, int((~odd).sum()), 32768, 16, 16, 100, n_threads=n_threads)
        b_buf, b_off, b_len, b_n = gen_zipf_blocks(seed + 1, int(odd.sum()), N.PBL_FMT_ROW, 16, 32768,
                                                   n_threads=n_threads)
        parts = [(a_buf, a_off, a_len), (b_buf, b_off, b_len)]
        src = np.where(odd, 1, 0)
        n_kv = a_n + b_n
    elif kind == "tail8":
        odd = ids % 8 == 7
        a_buf, a_off, a_len, a_n = gen_row_blocks(seed, int((~odd).sum()), 32768, 16, 16, 100, n_threads=n_threads)
        parts, n_kv = [(a_buf, a_off, a_len)], a_n
        src = np.zeros(n_blocks, np.int64)
        tails = np.nonzero(odd)[0]
        for k, bs in enumerate((2048, 4096, 8192)):
            sel = tails[k::3]
            t_buf, t_off, t_len, t_n = gen_row_blocks(seed + 1 + k, len(sel), bs, 16, 16, 100, n_threads=n_threads)
            parts.append((t_buf, t_off, t_len))
            src[sel] = 1 + k
            n_kv += t_n
    else:
        raise ValueError(kind)
    # the i-th block of each part, in batch order
    nth = np.zeros(n_blocks, np.int64)
    for p in range(len(parts)):
        m = src == p
        nth[m] = np.arange(int(m.sum()))
    lens = np.array([parts[p][2][i] for p, i in zip(src, nth)], np.uint32)
    slot = (lens.astype(np.uint64) + 7) // 8 * 8
    off = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(slot.sum()) + 16, np.uint8)
    for b in range(n_blocks):
        pb, po, _ = parts[src[b]]
        o = int(po[nth[b]])
        buf[int(off[b]): int(off[b]) + int(lens[b])] = pb[o: o + int(lens[b])]
    return buf, off, lens, int(n_kv)
