"""bench.py's multi-rank launcher on CPU: `bench.py --gpus N` (no WORLD_SIZE in
the environment) starts N ranks through torch.distributed.run as a child
process; each rank reads RANK / LOCAL_RANK / WORLD_SIZE, and rank 0 prints ONE
JSON line with n_gpus == N (--launch-check: gloo, no GPU touched)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_self_launch_yields_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["launch_check"]
    assert sorted(x[0] for x in d["ranks"]) == list(range(n))
    assert sorted(x[1] for x in d["ranks"]) == list(range(n))  # one local rank (GPU) per process
    assert all(x[2] == n for x in d["ranks"])
    if n > 1:
        assert d["parallelism"] == f"shard{n}+rccl_offset_concat"


def test_bench_multirank_step_on_gloo():
    """`bench.py --gpus 2 --dist-backend gloo` with no GPU: both ranks run the
    bench's own step -- its all-gather of per-rank totals and the rebase of the
    per-block bases (concat_step) -- and rank 0 prints one JSON line with
    n_gpus 2 and the concat checked against every rank's totals."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--blocks", "16", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["plumbing"] and d["concat_ok"] and d["steps"] == 3


@pytest.mark.parametrize("workload", ["row", "zipf"])
def test_bench_multirank_global_batch_is_byte_balanced(workload):
    """N > 1 cuts ONE global batch (world x --blocks blocks, content a function
    of the seed and the global block index) into contiguous byte-balanced ranges
    with shard.partition_blocks, and reports every rank's
    input bytes: here on gloo, checked against the partition of the global
    batch generated in one piece."""
    import numpy as np
    from pebble_amd.batch import gen_zipf_blocks
    from pebble_amd.rowblk import gen_row_blocks
    from pebble_amd.shard import partition_blocks
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--workload", workload, "--blocks", "24", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    lens = (gen_zipf_blocks(42, 48, 0, 16, 32768, n_threads=4)[2] if workload == "zipf"
            else gen_row_blocks(42, 48, 32768, 16, 16, 100, n_threads=4)[2])
    ranges = partition_blocks(lens, 2)
    c = d["config"]
    assert c["global_batch_blocks"] == 48 and c["shard_blocks"] == list(ranges[0])
    assert c["input_bytes_per_rank"] == [int(lens[s:e].astype(np.int64).sum()) for s, e in ranges]
    assert d["concat_ok"]
