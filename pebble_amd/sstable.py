"""Whole tables to decoded blocks on the device.

`Table` mirrors what sstable.Reader does at open and at iteration
(sstable/reader.go, table.go:298-404): read the footer, load the index, walk
its handles to the data blocks.  Every block step runs in libpebble_amd.so:

  footer          pbl_parse_footer (host: the last 61 bytes of the file)
  metaindex,      physical step (pbl_verify_checksums, pbl_decompress_blocks),
  properties      pbl_decode_batch with PBL_ROW_RAW_KEYS; the index type
                  ("rocksdb.block.based.table.index.type", a uvarint) decides
                  single- or two-level (table.go:156-160)
  index blocks    physical step, pbl_decode_batch, pbl_index_handles_row (row
                  formats); pbl_index_handles_col (columnar formats, one level)
  data blocks     the handles become a PhysBatch over the file bytes already
                  in HBM: checksums, decompression, then `batch.decode`

The index's handles never visit the host on the data path: they are device
arrays that become the next batch's offsets.  Row-format tables (LevelDB,
RocksDBv2, Pebblev1-v4) are read whole; for columnar tables (Pebblev5+) the
block-level index decode is here, their colblk metaindex/properties blocks are
not.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _native as N
from .batch import BlockBatch, DecodedBatch, DecodeError, _stream_handle, decode
from .physical import PhysBatch, decompress, verify_checksums

MAX_FOOTER_LEN = 61  # table.go maxFooterLen (Pebblev7+)
TWO_LEVEL_INDEX = 2  # table.go twoLevelIndex
INDEX_TYPE_PROP = b"rocksdb.block.based.table.index.type"
PROPERTIES_NAME = b"rocksdb.properties"


@dataclass
class Footer:
    table_format: int
    checksum_type: int
    metaindex: tuple
    index: tuple
    footer: tuple
    attributes: int

    @property
    def columnar(self) -> bool:
        return self.table_format >= N.PBL_TABLE_PEBBLEV1 + 4  # Pebblev5+ (format.go BlockColumnar)


def parse_footer(tail: bytes, file_size: int) -> Footer:
    """parseFooter over the last bytes of a file (pbl_parse_footer)."""
    f = N.FooterC()
    rc = N.lib().pbl_parse_footer(bytes(tail), len(tail), file_size, ctypes.byref(f))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_parse_footer: {N.STATUS_NAMES.get(rc, rc)}")
    return Footer(f.table_format, f.checksum_type, (f.metaindex_off, f.metaindex_len), (f.index_off, f.index_len),
                  (f.footer_off, f.footer_len), f.attributes)


@dataclass
class IndexHandles:
    handle_off: torch.Tensor  # int64 (u64) [n]
    handle_len: torch.Tensor  # int64 (u64) [n]
    props_off: torch.Tensor   # int64 [n]
    props_len: torch.Tensor   # int32 [n]
    blk_base: torch.Tensor    # int64 [n_blocks + 1]
    blk_status: torch.Tensor  # int32 [n_blocks]

    def c_struct(self) -> N.IndexOutC:
        return N.IndexOutC(self.handle_off.data_ptr(), self.handle_len.data_ptr(), self.props_off.data_ptr(),
                           self.props_len.data_ptr(), self.blk_base.data_ptr(), self.blk_status.data_ptr(),
                           self.handle_off.numel())

    @classmethod
    def allocate(cls, n_blocks: int, cap: int, device) -> "IndexHandles":
        e = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=device)  # noqa: E731
        return cls(e(cap, torch.int64), e(cap, torch.int64), e(cap, torch.int64), e(cap, torch.int32),
                   e(n_blocks + 1, torch.int64), e(n_blocks, torch.int32))

    def status(self) -> np.ndarray:
        return self.blk_status.cpu().numpy().view(np.uint32)

    def total(self, n_blocks: int) -> int:
        return int(self.blk_base[n_blocks].item())


def index_handles_row(decoded: DecodedBatch, n_blocks: int, stream=None) -> IndexHandles:
    """rowblk.IndexIter.BlockHandleWithProperties of every entry of decoded row
    index blocks (pbl_index_handles_row)."""
    n = int(decoded.read_totals().n_kv)
    out = IndexHandles.allocate(n_blocks, n, decoded.trailer.device)
    c = out.c_struct()
    o = decoded.c_struct()
    rc = N.lib().pbl_index_handles_row(ctypes.byref(o), n_blocks, ctypes.byref(c), _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_index_handles_row: {N.STATUS_NAMES.get(rc, rc)}")
    return out


def index_handles_col(batch: BlockBatch, cap: Optional[int] = None, stream=None) -> IndexHandles:
    """colblk.IndexIter handles of raw columnar index blocks
    (pbl_index_handles_col); re-runs once with the exact size on overflow."""
    cap = cap if cap is not None else max(1, batch.input_bytes() // 4)
    for _ in range(2):
        out = IndexHandles.allocate(batch.n_blocks, cap, batch.device)
        c = out.c_struct()
        b = batch.c_struct()
        rc = N.lib().pbl_index_handles_col(ctypes.byref(b), ctypes.byref(c), _stream_handle(stream))
        if rc != N.PBL_OK:
            raise DecodeError(f"pbl_index_handles_col: {N.STATUS_NAMES.get(rc, rc)}")
        tot = out.total(batch.n_blocks)
        if tot <= cap:
            return out
        cap = tot
    return out


def _uvarint(b: bytes, i: int = 0):
    x = s = 0
    while True:
        c = b[i]
        x |= (c & 0x7F) << s
        i += 1
        if c < 0x80:
            return x, i
        s += 7


class Table:
    """One SST whose bytes are resident on a device."""

    def __init__(self, data, device="cuda"):
        host = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        self.size = len(host)
        self.footer = parse_footer(host[max(0, self.size - MAX_FOOTER_LEN):].tobytes(), self.size)
        pad = np.zeros(self.size + 16, np.uint8)
        pad[: self.size] = host
        self.bytes = torch.from_numpy(pad).to(device)
        self.device = self.bytes.device

    # -- the physical step for any set of handles already on the device ----------
    def _blocks(self, off: torch.Tensor, length: torch.Tensor, fmt: int, flags: int = 0) -> BlockBatch:
        pb = PhysBatch(self.bytes, off.contiguous(), length.to(torch.int32).contiguous())
        st, _ = verify_checksums(pb, self.footer.checksum_type)
        if st.any():
            raise DecodeError(f"block checksum mismatch in {int((st != 0).sum())} block(s)")
        bb, st = decompress(pb, fmt, flags)
        if st.any():
            raise DecodeError(f"decompression failed: {sorted(set(N.STATUS_NAMES.get(int(x), x) for x in st))}")
        return bb

    def _handle_blocks(self, handles, fmt: int, flags: int = 0) -> BlockBatch:
        off = torch.tensor([h[0] for h in handles], dtype=torch.int64, device=self.device)
        ln = torch.tensor([h[1] for h in handles], dtype=torch.int64, device=self.device)
        return self._blocks(off, ln, fmt, flags)

    def _raw_kvs(self, handle) -> dict:
        """The KVs of one metadata row block (raw keys) as a host dict."""
        from .rowblk import kvs_of_block
        r = decode(self._handle_blocks([handle], N.PBL_FMT_ROW, N.PBL_ROW_RAW_KEYS)).to_host()
        if r["status_mask"]:
            raise DecodeError("metadata block corrupt")
        return {kv.user_key: kv.value for kv in kvs_of_block(r, 0)}

    def index_type(self) -> int:
        meta = self._raw_kvs(self.footer.metaindex)
        ph = meta.get(PROPERTIES_NAME)
        if ph is None:
            return 0
        off, i = _uvarint(ph)
        ln, _ = _uvarint(ph, i)
        props = self._raw_kvs((off, ln))
        v = props.get(INDEX_TYPE_PROP)
        return _uvarint(v)[0] if v else 0

    def data_block_handles(self) -> IndexHandles:
        """Every data block's handle, in table order, as device arrays."""
        if self.footer.columnar:
            return index_handles_col(self._handle_blocks([self.footer.index], N.PBL_FMT_ROW))
        two_level = self.index_type() == TWO_LEVEL_INDEX
        top = self._handle_blocks([self.footer.index], N.PBL_FMT_ROW)
        d = decode(top)
        h = index_handles_row(d, 1)
        if h.status().any():
            raise DecodeError("corrupt index block")
        if not two_level:
            return h
        n = h.total(1)
        lower = self._blocks(h.handle_off[:n], h.handle_len[:n], N.PBL_FMT_ROW)
        d2 = decode(lower)
        h2 = index_handles_row(d2, lower.n_blocks)
        if h2.status().any():
            raise DecodeError("corrupt lower-level index block")
        return h2

    def data_blocks(self, fmt: Optional[int] = None) -> BlockBatch:
        """The table's data blocks, checksum-verified and decompressed in HBM."""
        h = self.data_block_handles()
        n = int(h.blk_base[-1].item())
        fmt = fmt if fmt is not None else (N.PBL_FMT_COL_DEFAULT if self.footer.columnar else N.PBL_FMT_ROW)
        return self._blocks(h.handle_off[:n], h.handle_len[:n], fmt)

    def decode(self, fmt: Optional[int] = None) -> DecodedBatch:
        return decode(self.data_blocks(fmt))
