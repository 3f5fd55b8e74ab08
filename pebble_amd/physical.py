"""The physical-block step before decode, on the device.

Blocks as read from an SST file carry a 5-byte trailer, [compression indicator
u8][checksum LE32] (sstable/block/block.go:539-571).  `PhysBatch` holds such
blocks in HBM; `verify_checksums` is block.ValidateChecksum for a whole batch
(CRC32C / XXH64), `decompress` is Decompressor.DecompressedLen +
DecompressInto (snappy; uncompressed blocks are copied) producing a
`BlockBatch` ready for `batch.decode`.  All work runs in
libpebble_amd.so (pebble_amd/csrc/physical.hip).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as N
from .batch import BlockBatch, DecodeError, _stream_handle, varlen_hint


@dataclass
class PhysBatch:
    bytes: torch.Tensor      # uint8, the file bytes holding the blocks
    block_off: torch.Tensor  # int64 [n]: offset of each block
    block_len: torch.Tensor  # int32 [n]: block.Handle.Length (the trailer follows)
    flags: int = 0           # PBL_PHYS_* (PBL_PHYS_MINLZ_NATIVE: decode the MinLZ form)

    @property
    def n_blocks(self) -> int:
        return int(self.block_off.numel())

    @classmethod
    def from_host(cls, blob: np.ndarray, off, lens, device="cuda", flags: int = 0) -> "PhysBatch":
        b = np.zeros(len(blob) + 16, np.uint8)
        b[: len(blob)] = np.frombuffer(bytes(blob), np.uint8) if isinstance(blob, (bytes, bytearray)) else blob
        return cls(torch.from_numpy(b).to(device),
                   torch.from_numpy(np.ascontiguousarray(off, np.uint64).view(np.int64)).to(device),
                   torch.from_numpy(np.ascontiguousarray(lens, np.uint32).view(np.int32)).to(device), flags)

    def c_struct(self) -> N.PhysBatchC:
        return N.PhysBatchC(self.bytes.data_ptr(), self.block_off.data_ptr(), self.block_len.data_ptr(),
                            self.n_blocks, self.flags)


def verify_checksums(pb: PhysBatch, checksum_type: int, stream=None):
    """(status, computed) per block: PBL_OK or PBL_CORRUPT_CHECKSUM, and the
    checksum computed over the block bytes and the indicator byte."""
    dev = pb.bytes.device
    st = torch.empty(max(pb.n_blocks, 1), dtype=torch.int32, device=dev)
    comp = torch.empty(max(pb.n_blocks, 1), dtype=torch.int32, device=dev)
    c = pb.c_struct()
    rc = N.lib().pbl_verify_checksums(ctypes.byref(c), checksum_type, ctypes.c_void_p(st.data_ptr()),
                                      ctypes.c_void_p(comp.data_ptr()), _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_verify_checksums: {N.STATUS_NAMES.get(rc, rc)}")
    n = pb.n_blocks
    return st[:n].cpu().numpy().view(np.uint32), comp[:n].cpu().numpy().view(np.uint32)


def decompress(pb: PhysBatch, fmt: int = N.PBL_FMT_ROW, flags: int = 0, stream=None):
    """Decompress every block into a new device buffer (8-B aligned slots).
    Returns (BlockBatch of the decoded blocks, per-block status)."""
    dev = pb.bytes.device
    n = pb.n_blocks
    lens = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    st = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    c = pb.c_struct()
    lib = N.lib()
    rc = lib.pbl_decompressed_lengths(ctypes.byref(c), ctypes.c_void_p(lens.data_ptr()),
                                      ctypes.c_void_p(st.data_ptr()), _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_decompressed_lengths: {N.STATUS_NAMES.get(rc, rc)}")
    hl = lens[:n].cpu().numpy().view(np.uint32).astype(np.uint64)
    slot = (hl + 7) // 8 * 8
    off = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
    total = int(slot.sum()) if n else 0
    out = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    cap_t = torch.from_numpy(hl.astype(np.uint32).view(np.int32)).to(dev)
    rc = lib.pbl_decompress_blocks(ctypes.byref(c), ctypes.c_void_p(out.data_ptr()),
                                   ctypes.c_void_p(off_t.data_ptr()), ctypes.c_void_p(cap_t.data_ptr()),
                                   ctypes.c_void_p(lens.data_ptr()), ctypes.c_void_p(st.data_ptr()),
                                   _stream_handle(stream))
    if rc != N.PBL_OK:
        raise DecodeError(f"pbl_decompress_blocks: {N.STATUS_NAMES.get(rc, rc)}")
    status = st[:n].cpu().numpy().view(np.uint32).copy()
    return BlockBatch(out, off_t, lens[:n].clone(), fmt, flags | varlen_hint(hl.astype(np.uint32))), status
