"""Time corpus ingest on the GPU box: load_tokens (pre-split ids) and
load_text (the same corpus as a text file) for the bench corpus."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import swiftmpi_amd as sw  # noqa: E402
from swiftmpi_amd.synth import zipf_tokens  # noqa: E402

ids, off = zipf_tokens(17005207, 253854, 1000, seed=8)
keys = np.array([sw.bkdr("w%d" % i) for i in range(253854)], dtype=np.uint64)
with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "c.txt")
    t0 = time.perf_counter()
    words = np.array(["w%d" % i for i in range(253854)])
    with open(path, "w") as f:
        for l in range(len(off) - 1):
            f.write(" ".join(words[ids[off[l]:off[l + 1]]]) + "\n")
    print("write text %.1f s, %.0f MB" % (time.perf_counter() - t0, os.path.getsize(path) / 1e6), flush=True)
    for mode in ("tokens", "text"):
        t = sw.Table("w2v", dim=300, capacity=260000, dtype="f32", learning_rate=0.7)
        w = sw.Word2Vec(t, minibatch=5000, sample=1e-5, fp64_intermediates=False)
        t0 = time.perf_counter()
        if mode == "tokens":
            w.load_tokens(ids, off, keys)
        else:
            w.load_text(path)
        t1 = time.perf_counter()
        w.init()
        print("%s: ingest %.2f s, first pull %.2f s" % (mode, t1 - t0, time.perf_counter() - t1), flush=True)
        del w, t
