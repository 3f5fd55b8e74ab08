#!/usr/bin/env python3
"""Throughput of the physical-block step on config-2-shaped
data: 64 Ki x 32 KiB row blocks with 5-byte trailers.  The trailers' checksums
are produced by the device itself (a first verify pass reports `computed`,
which is written into the trailers; the timed passes then verify them all OK).
Snappy: the same blocks compressed on the host (pyarrow), decompressed on the
device.  Prints one JSON line.  Usage: bench_physical.py [n_blocks] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pebble_amd import _native as N  # noqa: E402
from pebble_amd.physical import PhysBatch, decompress, verify_checksums  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
buf, off, lens, _ = gen_row_blocks(42, nb, 32768, 16, 16, 100, n_threads=16)
stride = 32768 + 8
phys = np.zeros(nb * stride + 16, np.uint8)
pv = phys[: nb * stride].reshape(nb, stride)
pv[:, :32768] = buf[: nb * 32768].reshape(nb, 32768)
poff = np.arange(nb, dtype=np.uint64) * stride
res = {"blocks": nb, "block_bytes": int(lens.sum())}


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for name, ct in (("crc32c", N.PBL_CHECKSUM_CRC32C), ("xxhash64", N.PBL_CHECKSUM_XXHASH64)):
    pb = PhysBatch.from_host(phys, poff, lens)
    _, comp = verify_checksums(pb, ct)
    # write the device-computed checksums into the trailers (indicator 0 = none)
    host = pb.bytes.cpu().numpy()
    for i in range(nb):
        t = int(poff[i]) + int(lens[i])
        host[t + 1:t + 5] = np.frombuffer(int(comp[i]).to_bytes(4, "little"), np.uint8)
    pb = PhysBatch(torch.from_numpy(host).cuda(), pb.block_off, pb.block_len)
    st, _ = verify_checksums(pb, ct)
    assert not st.any()
    from pebble_amd.batch import _stream_handle
    import ctypes
    s_t = torch.empty(nb, dtype=torch.int32, device="cuda")
    c = pb.c_struct()
    sec = timed(lambda: N.lib().pbl_verify_checksums(ctypes.byref(c), ct, ctypes.c_void_p(s_t.data_ptr()), None,
                                                      _stream_handle(None)))
    res[name] = {"GB_per_s": round((int(lens.sum()) + nb) / sec / 1e9, 1), "ms": round(sec * 1e3, 3)}

import pyarrow as pa  # noqa: E402
codec = pa.Codec("snappy")
comp = [codec.compress(buf[int(o):int(o) + int(ln)].tobytes(), asbytes=True) for o, ln in zip(off, lens)]
cl = np.array([len(x) for x in comp], np.uint32)
coff = np.zeros(nb, np.uint64)
coff[1:] = np.cumsum((cl.astype(np.uint64) + 5 + 7) // 8 * 8)[:-1]
cbuf = np.zeros(int(coff[-1]) + int(cl[-1]) + 32, np.uint8)
for i, x in enumerate(comp):
    cbuf[int(coff[i]):int(coff[i]) + len(x)] = np.frombuffer(x, np.uint8)
    cbuf[int(coff[i]) + len(x)] = 1  # snappy indicator
pb = PhysBatch.from_host(cbuf, coff, cl)
bb, st = decompress(pb)
assert not st.any() and int(bb.block_len.to(torch.int64).sum()) == int(lens.sum())
assert np.array_equal(bb.blocks[: int(lens[0])].cpu().numpy(), buf[: int(lens[0])])
import ctypes  # noqa: E402
from pebble_amd.batch import _stream_handle  # noqa: E402
c = pb.c_struct()
o_len = torch.empty(nb, dtype=torch.int32, device="cuda")
o_st = torch.empty(nb, dtype=torch.int32, device="cuda")
cap = bb.block_len.clone()
sec = timed(lambda: N.lib().pbl_decompress_blocks(ctypes.byref(c), ctypes.c_void_p(bb.blocks.data_ptr()),
                                                  ctypes.c_void_p(bb.block_off.data_ptr()),
                                                  ctypes.c_void_p(cap.data_ptr()), ctypes.c_void_p(o_len.data_ptr()),
                                                  ctypes.c_void_p(o_st.data_ptr()), _stream_handle(None)))
res["snappy"] = {"decoded_GB_per_s": round(int(lens.sum()) / sec / 1e9, 1), "ms": round(sec * 1e3, 3),
                 "compressed_bytes": int(cl.sum()), "ratio": round(float(lens.sum()) / float(cl.sum()), 2)}
print(json.dumps(res), flush=True)
