"""In-tree build of libpebble_amd.so (hipcc, gfx950 only).

The library is built next to this file so that it travels with the repo
snapshot to the GPU box; nothing is installed into site-packages.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpebble_amd.so")
SOURCES = ["rowblk_decode.hip", "colblk_decode.hip", "transforms.hip", "physical.hip", "sstable.hip", "rowblk_writer.cpp", "colblk_writer.cpp", "zipf_gen.cpp"]
HEADERS = ["common.hip.h", "rowblk_general.hip.h", "rowblk_pipe.hip.h", "colblk_pipe.hip.h", "colblk_block.hip.h", os.path.join("..", "..", "include", "pebble_amd.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return False


DIAG_OUT = os.path.join(HERE, "libpebble_amd_diag.so")


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """Build libpebble_amd.so; `diag` builds the phase-stamp diagnostic variant
    (libpebble_amd_diag.so, -DPBL_STAMPS) used only by scripts/phase_stamps.py."""
    out = DIAG_OUT if diag else OUT
    if not force and not diag and not _stale():
        return OUT
    cmd = [HIPCC, *FLAGS, *(["-DPBL_STAMPS"] if diag else []), *[os.path.join(CSRC, s) for s in SOURCES],
           "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
