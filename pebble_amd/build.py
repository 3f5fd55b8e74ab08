"""In-tree build of libpebble_amd.so (hipcc, gfx950 only).

The library is built next to this file so that it travels with the repo
snapshot to the GPU box; nothing is installed into site-packages.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpebble_amd.so")
SOURCES = ["rowblk_decode.hip", "colblk_decode.hip", "transforms.hip", "physical.hip", "zstd.hip", "sstable.hip", "rowblk_writer.cpp", "colblk_writer.cpp", "zipf_gen.cpp", "data_iter.cpp"]
HEADERS = ["common.hip.h", "rowblk_general.hip.h", "rowblk_big.hip.h", "rowblk_pool.hip.h", "rowblk_wave.hip.h", "colblk_pipe.hip.h", "colblk_block.hip.h", "colblk_wave.hip.h", "zstd_dec.hip.h", "snappy_dec.hip.h", "minlz_dec.hip.h", os.path.join("..", "..", "include", "pebble_amd.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread"]


OBJ = os.path.join(HERE, ".obj")  # per-source objects (git- and gpurun-ignored)
DIAG_OUT = os.path.join(HERE, "libpebble_amd_diag.so")


def _newer(a: str, b: str) -> bool:
    return not os.path.exists(b) or os.path.getmtime(a) > os.path.getmtime(b)


def _stale(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    return any(_newer(os.path.join(CSRC, f), out) for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False, diag: bool = False, jobs: int = 8) -> str:
    """Build libpebble_amd.so: each source compiled to its own object (in
    parallel; only sources newer than their object, or any header newer), then
    one link.  `diag` builds the phase-stamp diagnostic variant
    (libpebble_amd_diag.so, -DPBL_STAMPS) used only by scripts/pipe_stamps.py."""
    out = DIAG_OUT if diag else OUT
    if not force and not _stale(out):
        return out
    tag = "diag" if diag else "rel"
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS)
    extra = ["-DPBL_STAMPS"] if diag else []
    cflags = [f for f in FLAGS if f != "-shared"]
    jobs_todo, objs = [], []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(OBJ, f"{os.path.splitext(src)[0]}.{tag}.o")
        objs.append(obj)
        if force or _newer(sp, obj) or hdr_t > os.path.getmtime(obj):
            jobs_todo.append(([HIPCC, *cflags, *extra, "-c", sp, "-o", obj + ".tmp"], obj))

    def compile_one(job):
        cmd, obj = job
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(obj + ".tmp", obj)

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(compile_one, jobs_todo))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
