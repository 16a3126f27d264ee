"""Host iteration-order fixture (SURVEY.md §7 hard part 1): the reference
orders its vocabulary (word2vec_global.h:385-444 `_local_keys`, a
std::unordered_set<size_t>), hence every vid, unigram slot and negative draw,
by libstdc++'s hash-set iteration, and LR's first-pull init order
(lr.cpp:157-...: std::unordered_set<unsigned>) the same way.  This script
records those orders ONCE, here in the build container where they were checked
against the reference, so a GPU box whose C++ runtime iterated
differently fails tests/test_order_fixture.py instead of passing against a
same-box oracle.

    python tests/golden/make_order_fixture.py

Inputs are regenerated from fixed seeds (numpy PCG64 streams are stable):
  w2v: conftest.zipf_corpus(5000 lines, vocab 20000, seed 77), BKDR keys "w<id>"
  lr:  tests/golden/lr_data.txt and a 4000-row Criteo-shaped text (synth.criteo seed 78, 2^14 features)
Outputs (tests/golden/order_fixture.npz): w2v_keys / w2v_counts (vid order),
w2v_starts (unigram run starts, table 1e8), lr_data_order, lr_criteo_order
(first-pull order)."""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def w2v_corpus(path):
    from conftest import zipf_corpus
    return zipf_corpus(path, 5000, 20000, seed=77)


def lr_criteo_text(path):
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(4000, seed=78, bits=14)
    with open(path, "w") as fh:
        for i in range(len(y)):
            a, b = int(off[i]), int(off[i + 1])
            fh.write("%g %s\n" % (y[i], " ".join("%d:%.9g" % (k, x) for k, x in zip(f[a:b], v[a:b]))))
    return path


def main():
    import oracle
    oracle.build()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        m = oracle.W2V(w2v_corpus(os.path.join(d, "c.txt")), 8, minibatch=100, table_size=int(1e8))
        out["w2v_keys"], out["w2v_counts"] = m.vocab()
        out["w2v_starts"] = m.table_starts()
        out["lr_data_order"] = oracle.LR(os.path.join(HERE, "lr_data.txt"), 200, 0.05).pull_order()
        out["lr_criteo_order"] = oracle.LR(lr_criteo_text(os.path.join(d, "lr.txt")), 255, 0.05).pull_order()
    np.savez_compressed(os.path.join(HERE, "order_fixture.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
