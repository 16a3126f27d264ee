import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import swiftmpi_amd as sw
from swiftmpi_amd.comm import Comm
from swiftmpi_amd.synth import criteo
torch.cuda.set_device(0)
B1 = 65537
nb = 10
y, off, f, v = criteo(B1 * nb, seed=3)
for sharded in (False, True):
    t = sw.Table("lr", capacity=1 << 23, dtype="f32", learning_rate=0.05, init="hash", seed=1, device=0)
    m = sw.LR(t, minibatch=65536, init_ref=False, profile=False, fast_sums=True, plan="none")
    m.load_csr(y, off, f, v)
    if sharded:
        comm = Comm.rccl(0, 1, port=29655)
        m.shard_comm(comm, frag_num=2000)
    m.init()
    m.train_batches(nb)
    m.sync()
    for rep in range(3):
        a = time.perf_counter()
        m.train_batches(40)
        b = time.perf_counter()
        m.sync()
        c = time.perf_counter()
        print("sharded=%d host issue %.1f us/step, total %.1f us/step" % (sharded, (b - a) / 40 * 1e6, (c - a) / 40 * 1e6), flush=True)
    m.close(); t.close()
