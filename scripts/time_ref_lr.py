"""Throughput of the reference's own lr.cpp, compiled unchanged against include/swiftmpi
(tests/cpp/_ref_apps/lr): one training pass over Criteo-shaped rows written in the reference's
text format, wall time of the binary (its host learn_instance + a pull and a push through the
HBM shard per minibatch).  Prints one JSON line."""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from swiftmpi_amd.synth import criteo  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 262148
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
d = tempfile.mkdtemp()
y, off, f, v = criteo(rows, seed=3)
data = os.path.join(d, "lr.txt")
with open(data, "w") as out:
    for r in range(rows):
        a, b = int(off[r]), int(off[r + 1])
        out.write("%g %s\n" % (y[r], " ".join("%d:%g" % (int(f[i]) & 0x7FFFFFFF, v[i]) for i in range(a, b))))
conf = os.path.join(d, "lr.conf")
with open(conf, "w") as c:
    c.write("[ worker ]\nminibatch: %d\nnthreads: 1\n[ server ]\ninitial_learning_rate: 0.05\nfrag_num: 1000\n"
            "out_param_prefix: %s\n" % (mb, os.path.join(d, "param")))
ref = os.path.join(ROOT, "tests", "cpp", "_ref_apps", "lr")
t0 = time.perf_counter()
r = subprocess.run([ref, "-mode", "train", "-config", conf, "-dataset", data, "-niters", "1"], capture_output=True,
                   text=True, timeout=900)
dt = time.perf_counter() - t0
assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
print(json.dumps({"what": "reference lr.cpp unchanged (host learn_instance, PS on the HBM shard)", "rows": rows,
                  "minibatch": mb, "features_per_row": float(off[-1]) / rows, "seconds": dt,
                  "examples_per_s": rows / dt}))
