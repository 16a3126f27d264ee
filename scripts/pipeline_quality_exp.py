import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np, socket, torch.distributed as dist
import swiftmpi_amd as lib
from swiftmpi_amd.synth import analogy_corpus, analogy_accuracy
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
path = "/tmp/an.txt"
qs = analogy_corpus(path, lines=2000)
words = sorted({w for q in qs for w in q})
from swiftmpi_amd.dist import ShardedWord2Vec
D = 32
for lr, B, ep in [(0.1, 100, 3), (0.05, 100, 5), (0.1, 400, 5), (0.7, 100, 3)]:
    res = []
    for pipeline in (False, True):
        t = lib.Table("w2v", dim=D, capacity=4096, dtype="f32", learning_rate=lr, init="hash", seed=5)
        sh = ShardedWord2Vec(t, pipeline=pipeline, window=5, negative=5, minibatch=B, sample=1e-3, unigram_size=10**7, fp64_intermediates=False)
        sh.load_text(path); sh.init(); sh.train(ep)
        vk, _ = sh.w.vocab(); keys, rows = sh.shard_rows()
        pos = {int(k): i for i, k in enumerate(keys)}
        rows = np.stack([rows[pos[int(k)]] for k in vk])
        idx = {int(k): i for i, k in enumerate(vk)}
        index = {w: idx[lib.bkdr(w)] for w in words}
        res.append(analogy_accuracy(rows[:, D:2 * D], index, qs, words))
    print("lr %.2f B %d ep %d  lockstep %.4f pipelined %.4f" % (lr, B, ep, res[0], res[1]), flush=True)
