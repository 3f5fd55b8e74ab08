"""Debug: decode a small synthetic row batch on cuda:0 and print per-block results next to the oracle's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from pebble_amd.batch import BlockBatch, decode  # noqa: E402
from pebble_amd.rowblk import gen_row_blocks  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
buf, off, lens, n = gen_row_blocks(7, nb, 32768, 16, 16, 100)
out = decode(BlockBatch.from_host(buf, off, lens, "cuda:0", 0, 0))
torch.cuda.synchronize()
g = out.to_host()
o = oracle.decode_batch(buf, off, lens, 0)
for k in ("n_kv", "key_bytes_total", "val_bytes_total", "n_restarts", "status_mask", "n_bad_blocks"):
    print(k, g[k], o[k])
print("n_slow", g["n_slow_blocks"])
print("status", g["blk_status"][:8], o["blk_status"][:8])
print("kvbase", g["blk_kv_base"][:8], o["blk_kv_base"][:8])
print("keybase", g["blk_key_base"][:8], o["blk_key_base"][:8])
print("rstbase", g["blk_rst_base"][:8], o["blk_rst_base"][:8])
print("ticket", out.workspace[:4].cpu().numpy().view(np.uint32))

if os.environ.get("PBL_LIB", "").endswith("_diag.so"):
    ws = out.workspace.cpu().numpy()
    st = ws[256 + 9 * nb * 8: 256 + 9 * nb * 8 + nb * 128].view(np.uint64).reshape(nb, 16)
    for b in range(nb):
        print("diag", b, [hex(int(x)) for x in st[b, :16]])
