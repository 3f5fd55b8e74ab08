"""The device zstd decoder's code (pebble_amd/csrc/zstd_dec.hip.h) run on the
host by scripts/zstd_emu.cpp -- 64 threads in lockstep at every wave primitive
-- against the oracle: h-zstd-compression-sst's blocks and facebook/zstd
frames, on both the LDS and the global-memory paths.  CPU-only: it checks the
same source the GPU build compiles, before the GPU runs it."""
import os
import random
import shutil
import subprocess

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("zemu") / "zstd_emu")
    subprocess.run(["g++", "-O1", "-std=c++20", "-pthread", os.path.join(ROOT, "scripts", "zstd_emu.cpp"), "-o", exe],
                   check=True)
    return exe


def run(emu, tmp_path, raw):
    i, o = tmp_path / "in.bin", tmp_path / "out.bin"
    i.write_bytes(raw)
    r = subprocess.run([emu, str(i), str(o)], capture_output=True, text=True, timeout=300)
    return o.read_bytes() if r.returncode == 0 else -r.returncode


def pebble_zstd(data: bytes, level: int) -> bytes:
    import pyarrow as pa
    n, pre = len(data), bytearray()
    while n >= 0x80:
        pre.append(n & 0x7F | 0x80)
        n >>= 7
    pre.append(n)
    return bytes(pre) + pa.Codec("zstd", compression_level=level).compress(data, asbytes=True)


def test_emulated_device_decoder_matches_oracle(emu, tmp_path):
    import json
    golden = os.path.join(ROOT, "tests", "golden")
    phys = json.load(open(os.path.join(golden, "physical.json")))
    blob = open(os.path.join(golden, "physical_blocks.bin"), "rb").read()
    for b in phys["h_zstd"]["blocks"][:6]:
        raw = blob[b["blob_off"]: b["blob_off"] + b["length"]]
        assert run(emu, tmp_path, raw) == oracle.zstd_block(raw)
    rng = random.Random(8)
    words = [rng.randbytes(rng.randrange(1, 12)) for _ in range(64)]

    def text(n):
        out = bytearray()
        while len(out) < n:
            out += rng.choice(words) if rng.random() < 0.8 else rng.randbytes(rng.randrange(1, 70))
        return bytes(out[:n])
    # (sizes past 28 KiB compressed / 36 KiB decoded take the global-memory path)
    for i, n in enumerate([1, 300, 2000, 9000, 30000, 36000, 45000, 30000, 2000]):
        data = [rng.randbytes, lambda k: b"z" * k, text][i % 3](n)
        raw = pebble_zstd(data, [1, 3, 19, -5][i % 4])
        assert run(emu, tmp_path, raw) == data, (i, n)
