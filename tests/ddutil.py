"""Helpers that read like the reference's datadriven iterator tests
(internal/itertest/datadriven.go, condensed output format)."""
from pebble_amd.rowblk import InternalKV


def fmt_kv(kv: InternalKV) -> str:
    return "." if kv is None else f"<{kv.user_key.decode()}:{kv.seq_num()}>"


def run_iter_cmds(it, cmds: str) -> str:
    out = []
    for line in cmds.strip().split("\n"):
        parts = line.split()
        op = parts[0]
        if op == "first":
            kv = it.First()
        elif op == "last":
            kv = it.Last()
        elif op == "next":
            kv = it.Next()
        elif op == "prev":
            kv = it.Prev()
        elif op == "seek-ge":
            kv = it.SeekGE(parts[1].encode())
        elif op == "seek-lt":
            kv = it.SeekLT(parts[1].encode())
        else:
            raise ValueError(op)
        out.append(fmt_kv(kv))
    return "".join(out)


def parse_ikeys(spec: str):
    """'a:1,b:2' -> [(b'a', seq 1), ...] (rowblk_iter_test.go:124-128)."""
    r = []
    for e in spec.strip().split(","):
        k, s = e.split(":")
        r.append((k.encode(), int(s)))
    return r
