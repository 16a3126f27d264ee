"""Round 6 (verdict r05 item 1): how many 128-B lines of the LR table a Criteo-shaped batch's
non-hot keys touch under two fid orders — first appearance by (batch, row tile), the library's, and
descending corpus count, the verdict's candidate — for [w | g2] rows (16 per line) and for a dense
weight array (32 per line).  CPU only: python scripts/lr_fid_order_sim.py [batches]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from swiftmpi_amd.synth import criteo
B1 = 65537
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10
y, off, f, v = criteo(B1 * nb, seed=3)
uk, inv, cnt = np.unique(f, return_inverse=True, return_counts=True)
V = len(uk); print("V", V, "nnz", len(f))
nhot = 512
ordc = np.lexsort((np.arange(V), -cnt))  # count desc, tie by vid
hot = ordc[:nhot]
# current: hot first, then by first appearance (batch, tile of 4096 rows) then key
rows_idx = np.repeat(np.arange(B1*nb), 39)
grp = np.full(V, 1<<62, dtype=np.int64)
g = (rows_idx // B1) * ((B1 + 4095)//4096) + (rows_idx % B1) // 4096
np.minimum.at(grp, inv, g)
ordp = np.lexsort((uk, grp))
def fids(order):
    fid = np.full(V, -1, np.int64)
    fid[hot] = np.arange(nhot)
    rest = order[~np.isin(order, hot)]
    fid[rest] = nhot + np.arange(len(rest))
    return fid
F = {"cur": fids(ordp), "count": fids(ordc)}
for name, fid in F.items():
    tot = {}
    for b in range(nb):
        s = inv[b*B1*39:(b+1)*B1*39]
        fb = fid[s]
        nh = fb[fb >= nhot]
        u = np.unique(nh)
        tot.setdefault("nonhot_rec", []).append(len(nh))
        tot.setdefault("uniq", []).append(len(u))
        tot.setdefault("lines_wg", []).append(len(np.unique(u // 16)))   # [w|g2] 8 B
        tot.setdefault("lines_w", []).append(len(np.unique(u // 32)))    # w only 4 B
        tot.setdefault("buckets", []).append(len(np.unique(u >> 12)))
    print(name, {k: int(np.mean(x)) for k, x in tot.items()})
