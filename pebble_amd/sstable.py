"""Whole tables to decoded blocks on the device.

`Table` mirrors what sstable.Reader does at open and at iteration
(sstable/reader.go:1160-1260, table.go:298-404): read the footer, the
metaindex and the properties, load the index, walk its handles to the data
blocks.  Every block step runs in libpebble_amd.so:

  footer          pbl_parse_footer (host: the last 61 bytes of the file)
  metaindex       physical step (pbl_verify_checksums, pbl_decompress_blocks),
                  then a colblk KeyValueBlock (pbl_kv_blocks) for Pebblev6+
                  (reader.go:536-545, layout.go:789-824) or a row block decoded
                  with PBL_ROW_RAW_KEYS before that (layout.go decodeMetaindex)
  properties      the same two block kinds, KeyValueBlock from Pebblev7 on
                  (reader.go:601-617).  "rocksdb.block.based.table.index.type"
                  (LE32, properties_gen.go:96-98) decides single- or two-level
                  (Properties.toAttributes, properties.go:221-223; a Pebblev7
                  footer's AttributeTwoLevelIndex bit must agree,
                  reader.go:1214-1221); "pebble.colblk.schema" picks the
                  columnar key schema ("crdb1" = cockroachkvs.KeySchema,
                  "DefaultKeySchema(<comparer>,<bundle>)" = colblk.DefaultKeySchema,
                  reader.go:1244-1254)
  index blocks    physical step, then pbl_index_handles_row (row formats, after
                  pbl_decode_batch) or pbl_index_handles_col (columnar formats);
                  two-level tables run the step twice, the top level's handles
                  becoming the second-level batch's offsets
  data blocks     the handles become a PhysBatch over the file bytes already
                  in HBM: checksums, decompression, then `batch.decode`

The index's handles never visit the host on the data path: they are device
arrays that become the next batch's offsets.  Only the metaindex and the
properties -- a few hundred bytes the reader also keeps on the host -- are
read back.
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
ATTRIBUTE_TWO_LEVEL_INDEX = 1 << 5  # attributes.go:13-18
INDEX_TYPE_PROP = b"rocksdb.block.based.table.index.type"
KEY_SCHEMA_PROP = b"pebble.colblk.schema"
PROPERTIES_NAME = b"rocksdb.properties"
VALUE_INDEX_NAME = b"pebble.value_index"


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
        return self.table_format >= N.PBL_TABLE_PEBBLEV5  # Pebblev5+ (format.go BlockColumnar)


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


@dataclass
class KvSlices:
    """colblk.KeyValueBlockDecoder KeyAt/ValueAt of every row of a batch of
    key-value blocks, as slices of the batch's bytes (pbl_kv_blocks)."""
    key_off: torch.Tensor     # int64 (u64) [n]
    key_len: torch.Tensor     # int32 [n]
    val_off: torch.Tensor     # int64 (u64) [n]
    val_len: torch.Tensor     # int32 [n]
    blk_base: torch.Tensor    # int64 [n_blocks + 1]
    blk_status: torch.Tensor  # int32 [n_blocks]

    def c_struct(self) -> N.KvOutC:
        return N.KvOutC(self.key_off.data_ptr(), self.key_len.data_ptr(), self.val_off.data_ptr(),
                        self.val_len.data_ptr(), self.blk_base.data_ptr(), self.blk_status.data_ptr(),
                        self.key_off.numel())

    def status(self) -> np.ndarray:
        return self.blk_status.cpu().numpy().view(np.uint32)


def kv_blocks(batch: BlockBatch, cap: Optional[int] = None, stream=None) -> KvSlices:
    """pbl_kv_blocks over a batch of colblk key-value blocks; re-runs once with
    the exact size on overflow."""
    cap = cap if cap is not None else max(1, batch.input_bytes() // 4)
    for _ in range(2):
        e = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=batch.device)  # noqa: E731
        out = KvSlices(e(cap, torch.int64), e(cap, torch.int32), e(cap, torch.int64), e(cap, torch.int32),
                       e(batch.n_blocks + 1, torch.int64), e(batch.n_blocks, torch.int32))
        c = out.c_struct()
        b = batch.c_struct()
        rc = N.lib().pbl_kv_blocks(ctypes.byref(b), ctypes.byref(c), _stream_handle(stream))
        if rc != N.PBL_OK:
            raise DecodeError(f"pbl_kv_blocks: {N.STATUS_NAMES.get(rc, rc)}")
        tot = int(out.blk_base[batch.n_blocks].item())
        if tot <= cap:
            return out
        cap = tot
    return out


def resolve_values(d: DecodedBatch, value_blocks: BlockBatch, stream=None) -> DecodedBatch:
    """pbl_resolve_values: every value-block handle of `d` replaced by the value
    it names in `value_blocks` (valueBlockFetcher.Fetch, valblk/reader.go:251-302).
    Returns a DecodedBatch sharing `d`'s keys and trailers with new values,
    per-block statuses and totals."""
    nb = d.n_blocks
    st = stream if stream is not None else torch.cuda.current_stream(d.trailer.device)
    cap = int(d.cap.val) + value_blocks.input_bytes() + 16
    for _ in range(2):
        with torch.cuda.stream(st):
            e = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=d.trailer.device)  # noqa: E731
            vo, vbytes = e(d.val_off.numel(), torch.int32), e(cap + 16, torch.uint8)
            base, bst = e(nb + 1, torch.int64), e(nb, torch.int32)
        c = N.ValueOutC(vo.data_ptr(), vbytes.data_ptr(), base.data_ptr(), bst.data_ptr(), cap)
        o = d.c_struct()
        vb = value_blocks.c_struct()
        rc = N.lib().pbl_resolve_values(ctypes.byref(o), nb, ctypes.byref(vb), ctypes.byref(c),
                                        ctypes.c_void_p(st.cuda_stream))
        if rc != N.PBL_OK:
            raise DecodeError(f"pbl_resolve_values: {N.STATUS_NAMES.get(rc, rc)}")
        st.synchronize()
        tot = int(base[nb].item()) if nb else 0
        if tot <= cap:
            break
        cap = tot
    t = d.read_totals()
    status = bst.cpu().numpy().view(np.uint32)
    mask = 0
    for x in set(status.tolist()):
        mask |= (1 << x) if x else 0
    t2 = N.TotalsC(t.n_kv, t.key_bytes, tot, t.n_restarts, mask, int((status != 0).sum()), t.n_slow_blocks, 0)
    totals = torch.frombuffer(bytearray(bytes(t2)), dtype=torch.uint8).to(d.trailer.device)
    from dataclasses import replace
    from .batch import Capacity
    cap2 = Capacity(d.cap.kv, d.cap.key, cap, d.cap.rst)
    return replace(d, val_off=vo, val_bytes=vbytes, blk_val_base=base, blk_status=bst, totals=totals, cap=cap2,
                   _host_totals=None)


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
        self._meta = None
        self._meta_raw = None
        self._props = None

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

    def _raw_kvs(self, handle, columnar: bool) -> dict:
        """The KVs of one metadata block as a host dict: a colblk KeyValueBlock
        (pbl_kv_blocks) or a row block with raw keys."""
        if columnar:
            bb = self._handle_blocks([handle], N.PBL_FMT_ROW)
            kv = kv_blocks(bb)
            st = kv.status()
            if st.any():
                raise DecodeError(f"metadata block corrupt ({N.STATUS_NAMES.get(int(st[0]), st[0])})")
            n = int(kv.blk_base[1].item())
            raw = bb.blocks.cpu().numpy().tobytes()
            ko, kl = kv.key_off[:n].cpu().tolist(), kv.key_len[:n].cpu().tolist()
            vo, vl = kv.val_off[:n].cpu().tolist(), kv.val_len[:n].cpu().tolist()
            return {raw[a:a + m]: raw[c:c + q] for a, m, c, q in zip(ko, kl, vo, vl)}
        from .rowblk import kvs_of_block
        r = decode(self._handle_blocks([handle], N.PBL_FMT_ROW, N.PBL_ROW_RAW_KEYS)).to_host()
        if r["status_mask"]:
            raise DecodeError("metadata block corrupt")
        return {kv.user_key: kv.value for kv in kvs_of_block(r, 0)}

    def metaindex(self) -> dict:
        """Block name -> (offset, length) (decodeColumnarMetaIndex, layout.go:789-824;
        row metaindex before Pebblev6).  The value-block index handle keeps only
        its block handle."""
        if self._meta is None:
            raw = self._raw_kvs(self.footer.metaindex, self.footer.table_format >= N.PBL_TABLE_PEBBLEV6)
            self._meta_raw = raw
            meta = {}
            for k, v in raw.items():
                try:
                    off, i = _uvarint(v)
                    ln, i = _uvarint(v, i)
                except IndexError:
                    raise DecodeError("pebble/table: invalid table (bad block handle)") from None
                if k != VALUE_INDEX_NAME and i != len(v):
                    raise DecodeError("pebble/table: invalid table (bad block handle)")
                meta[k] = (off, ln)
            self._meta = meta
        return self._meta

    def properties(self) -> dict:
        """Property name -> raw value bytes (decodePropertiesBlock, reader.go:601-617)."""
        if self._props is None:
            ph = self.metaindex().get(PROPERTIES_NAME)
            if ph is None and self.footer.table_format == N.PBL_TABLE_LEVELDB:
                self._props = {}  # (LevelDB tables written without one)
                return self._props
            if ph is None:
                raise DecodeError("did not read any value for the properties block in the meta index")
            self._props = self._raw_kvs(ph, self.footer.table_format >= N.PBL_TABLE_PEBBLEV7)
        return self._props

    def index_type(self) -> int:
        v = self.properties().get(INDEX_TYPE_PROP)
        if v is None:
            return 0
        if len(v) < 4:
            raise DecodeError("corrupt index type property")
        return int.from_bytes(v[:4], "little")  # binary.LittleEndian.Uint32 (properties_gen.go:98)

    def two_level(self) -> bool:
        two = self.index_type() == TWO_LEVEL_INDEX
        if self.footer.table_format >= N.PBL_TABLE_PEBBLEV7 and \
                bool(self.footer.attributes & ATTRIBUTE_TWO_LEVEL_INDEX) != two:
            raise DecodeError("pebble/table: attributes mismatch (two-level index)")
        return two

    def key_schema(self) -> int:
        """PBL_FMT_* of the data blocks: rowblk, or the columnar key schema the
        properties name (reader.go:1244-1254: an unknown schema is an error)."""
        if not self.footer.columnar:
            return N.PBL_FMT_ROW
        name = self.properties().get(KEY_SCHEMA_PROP, b"")
        if name == b"crdb1":
            return N.PBL_FMT_COL_CRDB1
        if name.startswith(b"DefaultKeySchema("):
            return N.PBL_FMT_COL_DEFAULT
        raise DecodeError(f"unknown key schema {name!r}")

    def data_block_handles(self) -> IndexHandles:
        """Every data block's handle, in table order, as device arrays."""
        two_level = self.two_level()
        top = self._handle_blocks([self.footer.index], N.PBL_FMT_ROW)
        if self.footer.columnar:
            h = index_handles_col(top)
        else:
            h = index_handles_row(decode(top), 1)
        if h.status().any():
            raise DecodeError("corrupt index block")
        if not two_level:
            return h
        n = h.total(1)
        lower = self._blocks(h.handle_off[:n], h.handle_len[:n], N.PBL_FMT_ROW)
        h2 = index_handles_col(lower) if self.footer.columnar else index_handles_row(decode(lower), lower.n_blocks)
        if h2.status().any():
            raise DecodeError("corrupt lower-level index block")
        return h2

    def data_blocks(self, fmt: Optional[int] = None) -> BlockBatch:
        """The table's data blocks, checksum-verified and decompressed in HBM.
        Row blocks of Pebblev3+ tables carry value prefixes
        (TableFormat.BlockHasValuePrefix; rowblk_iter.go hasValuePrefix)."""
        h = self.data_block_handles()
        n = int(h.blk_base[-1].item())
        fmt = fmt if fmt is not None else self.key_schema()
        flags = N.PBL_ROW_VALUE_PREFIX if (fmt == N.PBL_FMT_ROW and
                                           self.footer.table_format >= N.PBL_TABLE_PEBBLEV1 + 2) else 0
        return self._blocks(h.handle_off[:n], h.handle_len[:n], fmt, flags)

    def value_blocks(self) -> Optional[BlockBatch]:
        """The table's value blocks (metaindex "pebble.value_index": an
        IndexHandle, valblk.go:320-336; its rows through pbl_valblk_index), or
        None when it has none."""
        self.metaindex()
        raw = self._meta_raw.get(VALUE_INDEX_NAME)
        if raw is None:
            return None
        off, i = _uvarint(raw)
        ln, i = _uvarint(raw, i)
        if len(raw) != i + 3:
            raise DecodeError("pebble/table: invalid table (bad value blocks index handle)")
        nw, ow, lw = raw[i], raw[i + 1], raw[i + 2]
        vbi = self._handle_blocks([(off, ln)], N.PBL_FMT_ROW)
        vlen = int(vbi.block_len[0].item())
        rows = vlen // max(1, nw + ow + lw)
        ho = torch.empty(max(rows, 1), dtype=torch.int64, device=self.device)
        hl = torch.empty(max(rows, 1), dtype=torch.int64, device=self.device)
        n_st = torch.zeros(2, dtype=torch.int32, device=self.device)
        src = vbi.blocks.data_ptr() + int(vbi.block_off[0].item())
        rc = N.lib().pbl_valblk_index(src, vlen, nw, ow, lw, ho.data_ptr(), hl.data_ptr(), rows,
                                      n_st.data_ptr(), n_st.data_ptr() + 4, None)
        if rc != N.PBL_OK:
            raise DecodeError(f"pbl_valblk_index: {N.STATUS_NAMES.get(rc, rc)}")
        n, st = n_st.cpu().tolist()
        if st != N.PBL_OK:
            raise DecodeError("corrupt value block index")
        return self._blocks(ho[:n], hl[:n], N.PBL_FMT_ROW)

    def decode(self, fmt: Optional[int] = None, resolve: bool = True) -> DecodedBatch:
        """Decode every data block; with `resolve`, values stored in value blocks
        are fetched (pbl_resolve_values) as the table iterator does when it
        returns a value."""
        d = decode(self.data_blocks(fmt))
        if resolve:
            vb = self.value_blocks()
            if vb is not None:
                d = resolve_values(d, vb)
        return d
