"""Row-block generators shared by the HideObsoletePoints tests (host only)."""
import random

from pebble_amd.rowblk import Writer, make_trailer


def mvcc_block(rng: random.Random, n: int = 200, ri: int = 16, vp: bool = False, share_trailer: bool = True):
    """Versions of user keys (1-4 per key, descending seqnums, kinds SET / DEL /
    SINGLEDEL, about a third obsolete), the shared prefix allowed into the
    trailer when `share_trailer` (a writer sharing whole internal keys, as
    LevelDB-era writers did): consecutive versions then share the kind byte."""
    w = Writer(ri)
    i = 0
    base = rng.randrange(1 << 20)
    while i < n:
        uk = b"user%08d" % (base + i) + bytes(rng.randint(97, 122) for _ in range(rng.randint(0, 6)))
        seq = rng.randrange(1 << 40) + 1000
        kind = rng.choice([1, 1, 0, 7])
        for v in range(rng.randint(1, 4)):
            if rng.random() < 0.3:
                kind = rng.choice([1, 0, 7])
            seq -= rng.randint(1, 3)
            tr = make_trailer(seq, kind)
            val = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 30])))
            obs = rng.random() < 0.35
            msk = len(uk) + 8 if share_trailer else len(uk)
            if vp and kind == 1:
                w.add_with_optional_value_prefix(uk, tr, obs, val, msk, True, rng.choice([0x00, 0x80, 0xC0]), False)
            else:
                w.add_with_optional_value_prefix(uk, tr, obs, val, msk, False, 0, False)
            i += 1
    return w.finish()
