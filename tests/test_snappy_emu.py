"""The device snappy decoder's code (pebble_amd/csrc/snappy_dec.hip.h: element
walk, copy-chain resolution by pointer jumping, literal and copy phases) run on
the host by scripts/snappy_emu.cpp -- 64 threads in lockstep at every wave
primitive -- against the oracle: hamlet-sst's snappy blocks, config-2-shaped
blocks and text-like blocks.  CPU-only: it checks the source the GPU build
compiles before the GPU runs it."""
import os
import random
import subprocess

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no clang++")
    exe = str(tmp_path_factory.mktemp("semu") / "snappy_emu")
    subprocess.run([CLANG, "-O1", "-std=c++20", "-pthread", os.path.join(ROOT, "scripts", "snappy_emu.cpp"), "-o", exe],
                   check=True)
    return exe


def run(emu, tmp_path, raw):
    i, o = tmp_path / "in.bin", tmp_path / "out.bin"
    i.write_bytes(raw)
    r = subprocess.run([emu, str(i), str(o)], capture_output=True, text=True, timeout=300)
    return o.read_bytes() if r.returncode == 0 else None


def test_emulated_snappy_decoder_matches_oracle(emu, tmp_path):
    import json
    import pyarrow as pa
    golden = os.path.join(ROOT, "tests", "golden")
    phys = json.load(open(os.path.join(golden, "physical.json")))
    blob = open(os.path.join(golden, "physical_blocks.bin"), "rb").read()
    for b in phys["hamlet_snappy"]["blocks"][:6]:
        raw = blob[b["blob_off"]: b["blob_off"] + b["length"]]
        assert run(emu, tmp_path, raw) == oracle.snappy_decode(raw)
    from pebble_amd.rowblk import gen_row_blocks
    buf, off, lens, _ = gen_row_blocks(7, 2, 32768, 16, 16, 100, n_threads=1)
    rng = random.Random(3)
    words = [rng.randbytes(rng.randrange(1, 10)) for _ in range(300)]
    text = b" ".join(rng.choice(words) for _ in range(6000))[:30000]
    # the bench's text corpus kind (a 512-word vocabulary of 2-8 characters):
    # most copies' sources span two elements and run in snappy4's phase 5
    vocab = [bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789") for _ in range(rng.randrange(2, 9))) + b" "
             for _ in range(512)]
    words = b"".join(rng.choice(vocab) for _ in range(8000))[:32768]
    for data in [bytes(buf[int(off[0]):int(off[0]) + int(lens[0])]), text, words, b"ab" * 9000, rng.randbytes(20000),
                 rng.randbytes(32768)]:  # (the last one compresses to more than 32 KiB)
        raw = pa.Codec("snappy").compress(data, asbytes=True)
        assert run(emu, tmp_path, raw) == data


def _uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_emulated_walk_capacity_and_overwrite_paths(emu, tmp_path, monkeypatch):
    """Blocks of 1-byte literals (more elements than one snappy4 round holds,
    every output byte its own element), the scalar-walk decode of snappy2
    (EMU_NO_WALK) and a corrupt block the walk rejects."""
    rng = random.Random(11)
    for d_len in (200, 4000):
        data = rng.randbytes(d_len)
        raw = _uvarint(d_len) + b"".join(bytes([0, c]) for c in data)  # 1-byte literals
        assert oracle.snappy_decode(raw) == data
        assert run(emu, tmp_path, raw) == data
    import pyarrow as pa
    text = b" ".join(rng.choice([b"alpha", b"beta", b"gamma", b"delta"]) for _ in range(5000))
    raw = pa.Codec("snappy").compress(text, asbytes=True)
    monkeypatch.setenv("EMU_NO_WALK", "1")
    assert run(emu, tmp_path, raw) == text
    # corrupt: a copy reaching before the output start
    bad = _uvarint(100) + bytes([0, 65]) + bytes([1 | (7 << 2), 9]) + bytes([0, 66]) * 10
    assert run(emu, tmp_path, bad) is None
