"""Device checksums and decompression (pebble_amd/csrc/physical.hip) against
the oracle and the reference's own SSTs: every stored CRC32C of the three test
files verifies on the device, corrupted blocks are caught, snappy blocks
decompress on the device and decode to exactly h.txt's KVs, XXH64 and snappy
agree with the oracle on random inputs (single-wave LDS path and the >32 KiB
global path), corrupt snappy is rejected; zstd blocks (h-zstd-compression-sst)
decompress on the device to exactly h.txt's KVs, and random zstd frames made
by facebook/zstd (pyarrow's codec) at levels -5..19 decode to the oracle's
bytes on both the LDS and the global path, corrupt ones as the oracle says."""
import os
import random

import numpy as np
import pytest

import oracle
from pebble_amd import _native as N
from pebble_amd.batch import decode
from pebble_amd.physical import PhysBatch, decompress, verify_checksums
from pebble_amd.rowblk import kvs_of_block

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _fixtures():
    import json
    with open(os.path.join(GOLDEN, "physical.json")) as f:
        phys = json.load(f)
    blob = np.fromfile(os.path.join(GOLDEN, "physical_blocks.bin"), np.uint8)
    return phys, blob


PHYS, BLOB = _fixtures()


def file_batch(name, blob=BLOB):
    bl = PHYS[name]["blocks"]
    return PhysBatch.from_host(blob, [b["blob_off"] for b in bl], [b["length"] for b in bl])


def pack_phys(blocks, checksum, rng=None, indicator=0):
    """[block][indicator][checksum LE32] at ragged offsets."""
    rng = rng or random.Random(0)
    buf, off, lens, pos = bytearray(), [], [], 0
    for bk in blocks:
        pos += rng.randrange(0, 8)
        buf += bytes(pos - len(buf))
        ind = indicator if isinstance(indicator, int) else indicator(bk)
        body = bytes(bk) + bytes([ind])
        off.append(pos)
        lens.append(len(bk))
        buf += body + int(checksum(body)).to_bytes(4, "little")
        pos = len(buf)
    return np.frombuffer(bytes(buf), np.uint8), off, lens


def test_stored_crc32c_checksums_verify():
    for name in PHYS:
        st, comp = verify_checksums(file_batch(name), N.PBL_CHECKSUM_CRC32C)
        assert list(st) == [0] * len(st), name
        assert list(comp) == [b["checksum"] for b in PHYS[name]["blocks"]], name


def test_corrupted_blocks_caught():
    blob = BLOB.copy()
    bl = PHYS["hamlet_snappy"]["blocks"] + PHYS["h_zstd"]["blocks"]
    rng = random.Random(3)
    bad = set()
    for i, b in enumerate(bl):
        if i % 3 == 0:
            pos = rng.choice([0, b["length"] - 1, b["length"], rng.randrange(b["length"])])  # incl. the indicator
            blob[b["blob_off"] + pos] ^= 1 << rng.randrange(8)
            bad.add(i)
    pb = PhysBatch.from_host(blob, [b["blob_off"] for b in bl], [b["length"] for b in bl])
    st, _ = verify_checksums(pb, N.PBL_CHECKSUM_CRC32C)
    assert [i for i, s in enumerate(st) if s == N.PBL_CORRUPT_CHECKSUM] == sorted(bad)
    assert all(s in (0, N.PBL_CORRUPT_CHECKSUM) for s in st)


@pytest.mark.parametrize("kind", ["crc32c", "xxhash64"])
def test_random_blocks_checksums(kind):
    rng = random.Random(11)
    sizes = [0, 1, 2, 3, 4, 5, 7, 31, 32, 33, 63, 64, 255, 256, 257, 4095, 4096, 65536, 200_001]
    sizes += [rng.randrange(0, 40_000) for _ in range(300)]
    blocks = [rng.randbytes(n) for n in sizes]
    fn = (lambda b: oracle.block_checksum(1, b)) if kind == "crc32c" else oracle.xxhash64_checksum
    ct = N.PBL_CHECKSUM_CRC32C if kind == "crc32c" else N.PBL_CHECKSUM_XXHASH64
    buf, off, lens = pack_phys(blocks, fn, rng)
    st, comp = verify_checksums(PhysBatch.from_host(buf, off, lens), ct)
    assert list(st) == [0] * len(blocks)
    for i in range(0, len(blocks), 7):  # a corrupted copy of every 7th block
        b = bytearray(buf[off[i]: off[i] + lens[i] + 5])
        b[rng.randrange(len(b) - 4)] ^= 0x80
        pb = PhysBatch.from_host(np.frombuffer(bytes(b), np.uint8), [0], [lens[i]])
        s, c = verify_checksums(pb, ct)
        assert s[0] == N.PBL_CORRUPT_CHECKSUM and c[0] == fn(bytes(b[: lens[i] + 1]))


def test_unsupported_checksum_types():
    pb = file_batch("h_no_compression")
    for ct in (N.PBL_CHECKSUM_NONE, N.PBL_CHECKSUM_XXHASH, 9):
        with pytest.raises(Exception, match="UNSUPPORTED"):
            verify_checksums(pb, ct)


def hamlet_kvs(batch):
    r = decode(batch).to_host()
    assert r["status_mask"] == 0
    kvs = []
    for b in range(batch.n_blocks):
        kvs += kvs_of_block(r, b)
    return [(kv.user_key.decode(), kv.value.decode()) for kv in kvs]


@pytest.mark.parametrize("name", ["hamlet_snappy", "h_no_compression"])
def test_decompress_then_decode_is_hamlet(name, golden):
    bb, st = decompress(file_batch(name))
    assert list(st) == [0] * bb.n_blocks
    assert list(bb.block_len.cpu().numpy()) == [b["decompressed_len"] for b in PHYS[name]["blocks"]]
    assert hamlet_kvs(bb) == [tuple(x) for x in golden["hamlet_kvs"]]


@pytest.mark.parametrize("name", ["h_zstd"])
def test_zstd_blocks_decode_to_hamlet(name, golden):
    bb, st = decompress(file_batch(name))
    assert list(st) == [0] * bb.n_blocks
    assert list(bb.block_len.cpu().numpy()) == [b["decompressed_len"] for b in PHYS[name]["blocks"]]
    assert hamlet_kvs(bb) == [tuple(x) for x in golden["hamlet_kvs"]]


def zstd_block(raw: bytes, level: int) -> bytes:
    """Pebble's zstd block: uvarint decoded length + a zstd frame (zstd_cgo.go:45-66)."""
    import pyarrow as pa
    n, pre = len(raw), bytearray()
    while n >= 0x80:
        pre.append(n & 0x7F | 0x80)
        n >>= 7
    pre.append(n)
    return bytes(pre) + pa.Codec("zstd", compression_level=level).compress(raw, asbytes=True)


def zstd_corpus(rng, i, n):
    if i % 4 == 0:
        return rng.randbytes(n)
    if i % 4 == 1:
        return bytes([rng.choice(b"xy")]) * n
    return compressible(rng, n)


def test_zstd_random_frames_lds_and_global_paths():
    rng = random.Random(21)
    sizes = [1, 2, 5, 64, 65, 1000, 4096, 28000, 32768, 36864, 36865, 40_000, 131_072, 300_000]
    sizes += [rng.randrange(1, 37_000) for _ in range(120)]
    raw = [zstd_corpus(rng, i, n) for i, n in enumerate(sizes)]
    comp = [zstd_block(r, rng.choice([-5, 1, 3, 9, 19])) for r in raw]
    buf, off, lens = pack_phys(comp, lambda b: 0, rng, indicator=7)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    assert list(st) == [0] * len(comp)
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, want in enumerate(raw):
        assert bl[i] == len(want), i
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == want, i
        if i < 30:
            assert oracle.zstd_block(comp[i]) == want


def test_zstd_mixed_with_snappy_and_raw():
    rng = random.Random(22)
    raw = [compressible(rng, rng.randrange(1, 30_000)) for _ in range(60)]
    blocks, inds = [], []
    for i, r in enumerate(raw):
        k = i % 3
        blocks.append(zstd_block(r, 3) if k == 0 else snappy(r) if k == 1 else r)
        inds.append(7 if k == 0 else 1 if k == 1 else 0)
    it = iter(inds)
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=lambda b: next(it))
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    assert list(st) == [0] * len(blocks)
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, want in enumerate(raw):
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == want, i


def test_zstd_batch_path_and_fallback_in_one_batch():
    """Blocks the batch path plans (one frame, one compressed block) next to
    blocks it leaves to zstd_kernel (two frames, a skippable frame first, a
    raw zstd block, more than 36 KiB decoded): every one decodes exactly."""
    import pyarrow as pa
    rng = random.Random(24)

    def uv(n):
        pre = bytearray()
        while n >= 0x80:
            pre.append(n & 0x7F | 0x80)
            n >>= 7
        pre.append(n)
        return bytes(pre)

    c = pa.Codec("zstd", compression_level=3)
    raw, comp = [], []
    for i in range(96):
        k = i % 6
        r = compressible(rng, rng.randrange(2000, 30_000))
        if k == 1:  # two frames
            a, b = r[: len(r) // 2], r[len(r) // 2:]
            comp.append(uv(len(r)) + c.compress(a, asbytes=True) + c.compress(b, asbytes=True))
        elif k == 2:  # a skippable frame, then the frame
            skip = (0x184D2A50).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"pebbl"
            comp.append(uv(len(r)) + skip + c.compress(r, asbytes=True))
        elif k == 3:  # incompressible: a raw zstd block
            r = rng.randbytes(rng.randrange(100, 20_000))
            comp.append(zstd_block(r, 3))
        elif k == 4:  # past the batch path's 36 KiB window
            r = compressible(rng, rng.randrange(36_865, 60_000))
            comp.append(zstd_block(r, 3))
        else:
            comp.append(zstd_block(r, rng.choice([1, 3, 9])))
        raw.append(r)
    buf, off, lens = pack_phys(comp, lambda b: 0, rng, indicator=7)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    assert list(st) == [0] * len(comp)
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, want in enumerate(raw):
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == want, i
        if i < 12:
            assert oracle.zstd_block(comp[i]) == want, i


def test_zstd_corrupt_matches_oracle():
    rng = random.Random(23)
    blocks = []
    for i in range(80):
        r = zstd_corpus(rng, i % 3 + 1, rng.randrange(1, 30_000))
        b = bytearray(zstd_block(r, rng.choice([1, 3, 19])))
        m = i % 5
        if m == 0:
            b = b[: rng.randrange(1, len(b))]                  # truncated
        elif m == 1:
            b[rng.randrange(4, len(b))] ^= 1 << rng.randrange(8)  # one bit flipped past the length
        elif m == 2:
            b = bytearray(b"\xff" * 11)                        # unterminated length varint
        elif m == 3:
            b[0] = (b[0] + 1) & 0x7F if b[0] < 0x80 else b[0]   # wrong decoded length
        blocks.append(bytes(b))
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=7)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, b in enumerate(blocks):
        want = oracle.zstd_block(b)
        if isinstance(want, int):
            assert st[i] in (N.PBL_CORRUPT_COMPRESSION, N.PBL_UNSUPPORTED), (i, st[i], want)
        else:
            assert st[i] == 0 and bytes(out[bo[i]: bo[i] + bl[i]]) == want, i


def snappy(b: bytes) -> bytes:
    import pyarrow as pa
    return pa.Codec("snappy").compress(b, asbytes=True)


def compressible(rng, n):
    words = [rng.randbytes(rng.randrange(1, 12)) for _ in range(64)]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words) if rng.random() < 0.8 else rng.randbytes(rng.randrange(1, 70))
    return bytes(out[:n])


def test_snappy_random_blocks_lds_and_global_paths():
    rng = random.Random(5)
    sizes = [0, 1, 2, 5, 64, 65, 1000, 32767, 32768, 32769, 40_000, 131_072, 300_000]
    sizes += [rng.randrange(0, 33_000) for _ in range(200)]
    raw = [compressible(rng, n) if i % 4 else rng.randbytes(n) for i, n in enumerate(sizes)]
    # runs: long overlapping copies (offset 1..8)
    raw += [bytes([i % 251]) * 5000 + bytes(range(7)) * 3000 for i in range(4)]
    comp = [snappy(b) for b in raw]
    ind = {c: 1 for c in comp}
    blocks = comp + raw[:20]  # the uncompressed copies (indicator 0)
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=lambda b: 1 if b in ind else 0)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    assert list(st) == [0] * len(blocks)
    out = bb.blocks.cpu().numpy()
    bo = bb.block_off.cpu().numpy()
    bl = bb.block_len.cpu().numpy()
    for i, want in enumerate(raw + raw[:20]):
        assert bl[i] == len(want), i
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == want, i
    for i, c in enumerate(comp[:40]):
        assert oracle.snappy_decode(c) == raw[i]


def test_snappy_corrupt_matches_oracle():
    rng = random.Random(9)
    good = [snappy(compressible(rng, rng.randrange(1, 50_000))) for _ in range(40)]
    blocks = []
    for g in good:
        b = bytearray(g)
        m = rng.randrange(4)
        if m == 0:
            b = b[: rng.randrange(1, len(b))]            # truncated
        elif m == 1:
            b[rng.randrange(3, len(b))] = rng.randrange(256)  # one byte changed (past the length)
        elif m == 2:
            b = bytearray(b"\xff" * 11)                     # unterminated length varint
        else:
            b = bytearray(b"\x10\x05\x00")                  # copy before any output
        blocks.append(bytes(b))
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=1)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens))
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, b in enumerate(blocks):
        want = oracle.snappy_decode(b)
        if want is None:
            assert st[i] in (N.PBL_CORRUPT_COMPRESSION,), (i, st[i])
        else:
            assert st[i] == 0 and bytes(out[bo[i]: bo[i] + bl[i]]) == want, i


# ---- MinLZ (indicator 8) ---------------------------------------------------------
def test_minlz_snappy_form_decodes_to_hamlet(golden):
    """minlz_test.go:31-36: a MinLZ decompressor decodes the Snappy fallback's
    output — the reference's snappy hamlet blocks relabelled indicator 8."""
    blob = BLOB.copy()
    for b in PHYS["hamlet_snappy"]["blocks"]:
        blob[b["blob_off"] + b["length"]] = N.PBL_COMPRESSION_MINLZ
    bb, st = decompress(file_batch("hamlet_snappy", blob))
    assert list(st) == [0] * bb.n_blocks
    assert list(bb.block_len.cpu().numpy()) == [b["decompressed_len"] for b in PHYS["hamlet_snappy"]["blocks"]]
    assert hamlet_kvs(bb) == [tuple(x) for x in golden["hamlet_kvs"]]


def test_minlz_random_blocks_lds_and_global_paths():
    """The MinLZ form (parity unpinned: the oracle's restatement of the format,
    oracle/minlz_oracle.c) on the device, every op form and the stored form,
    blocks past the 32 KiB stage on the global path."""
    rng = random.Random(31)
    sizes = [0, 1, 2, 5, 64, 65, 1000, 32767, 32768, 32769, 40_000, 131_072, 300_000]
    sizes += [rng.randrange(0, 33_000) for _ in range(150)]
    raw = []
    for i, n in enumerate(sizes):
        k = i % 5
        raw.append(rng.randbytes(n) if k == 0 else bytes([rng.randrange(3)]) * n if k == 1 else compressible(rng, n))
    far = rng.randbytes(70_000)
    raw += [far + rng.randbytes(50) + far[:5000], bytes(rng.randrange(3) for _ in range(40_000))]
    comp = [oracle.minlz_encode(r, i % 16) for i, r in enumerate(raw)]
    comp += [snappy(r) for r in raw[:30]]  # the Snappy form under indicator 8
    want = raw + raw[:30]
    buf, off, lens = pack_phys(comp, lambda b: 0, rng, indicator=N.PBL_COMPRESSION_MINLZ)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens, flags=N.PBL_PHYS_MINLZ_NATIVE))
    assert list(st) == [0] * len(comp)
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, w in enumerate(want):
        assert bl[i] == len(w), i
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == w, i
        assert oracle.minlz_decode(comp[i]) == w


def test_minlz_corrupt_matches_oracle():
    rng = random.Random(32)
    blocks = []
    for i in range(120):
        r = compressible(rng, rng.randrange(1, 40_000))
        b = bytearray(oracle.minlz_encode(r, rng.randrange(8)))
        m = i % 6
        if m == 0:
            b = b[: rng.randrange(1, len(b))]                      # truncated
        elif m == 1:
            b[rng.randrange(3, len(b))] ^= 1 << rng.randrange(8)  # one bit flipped past the header
        elif m == 2:
            b = bytearray(b"\x00" + b"\xff" * 11)                 # unterminated length varint
        elif m == 3:
            b[1] = (b[1] + 1) & 0x7F if b[1] < 0x80 else b[1]     # wrong decoded length
        elif m == 4:
            b = bytearray(b"\x00\x05\x05\x00")                    # copy before any output
        blocks.append(bytes(b))
    blocks += [b"", b"\x00", b"\x00\x00", b"\x00\x00abc", b"\x00\x01\x08ab"]
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=N.PBL_COMPRESSION_MINLZ)
    bb, st = decompress(PhysBatch.from_host(buf, off, lens, flags=N.PBL_PHYS_MINLZ_NATIVE))
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, b in enumerate(blocks):
        want = oracle.minlz_decode(b)
        if want is None:
            assert st[i] == N.PBL_CORRUPT_COMPRESSION, (i, st[i])
        else:
            assert st[i] == 0 and bytes(out[bo[i]: bo[i] + bl[i]]) == want, i


def test_minlz_mixed_with_other_codecs():
    rng = random.Random(33)
    raw = [compressible(rng, rng.randrange(1, 30_000)) for _ in range(80)]
    blocks, inds = [], []
    for i, r in enumerate(raw):
        k = i % 4
        blocks.append(zstd_block(r, 3) if k == 0 else snappy(r) if k == 1 else oracle.minlz_encode(r, 3) if k == 2 else r)
        inds.append(7 if k == 0 else 1 if k == 1 else 8 if k == 2 else 0)
    it = iter(inds)
    buf, off, lens = pack_phys(blocks, lambda b: 0, rng, indicator=lambda b: next(it))
    bb, st = decompress(PhysBatch.from_host(buf, off, lens, flags=N.PBL_PHYS_MINLZ_NATIVE))
    assert list(st) == [0] * len(blocks)
    # without the opt-in flag the MinLZ-form blocks are left to the host
    # (PBL_UNSUPPORTED); every other block decodes the same
    bb0, st0 = decompress(PhysBatch.from_host(buf, off, lens))
    out0, bo0, bl0 = bb0.blocks.cpu().numpy(), bb0.block_off.cpu().numpy(), bb0.block_len.cpu().numpy()
    for i, want in enumerate(raw):
        if inds[i] == 8:
            assert st0[i] == N.PBL_UNSUPPORTED, i
        else:
            assert st0[i] == 0 and bytes(out0[bo0[i]: bo0[i] + bl0[i]]) == want, i
    out, bo, bl = bb.blocks.cpu().numpy(), bb.block_off.cpu().numpy(), bb.block_len.cpu().numpy()
    for i, want in enumerate(raw):
        assert bytes(out[bo[i]: bo[i] + bl[i]]) == want, i
