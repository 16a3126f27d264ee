"""CPU attribution of the word2vec intermediates' rounding (no GPU).

Runs the oracle (the reference's CBOW-NS arithmetic, fp32 row storage) with
one rounding of the GPU kernels emulated at a time (oracle/swps_oracle.cpp
orc_set_diag_round) and prints the full-array relative distance from the
unrounded oracle, on the corpora of tests/test_bench_shape_gpu.py:

    python scripts/diag_bfp.py            # the table in swps_w2v_bfp.h

bits: 1 neu1 -> fp32, 2 neu1e -> fp32, 4 128-record chunk partials -> fp32,
8 mean -> fp32 (3 | 4 | 8 = fast mode's roundings, 15); 16: bits 1/2 keep a
bf16 residual; 32: an int16 residual per element; 64: int16 residual with one
scale per row (+128: int8); 256 / 512: block floating point rows with int32 /
int40 mantissas (BFP32 / BFP40); 1024: int24 mantissas (BFP24)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from test_bench_shape_gpu import CFG, corpus, rel_err  # noqa: E402

MODES = [("fast (fp32)", 15), ("BFP32", 259), ("fp32 + int16/row", 67 | 2 | 1), ("BFP40", 515), ("BFP24", 1027)]
if os.environ.get("DIAG_MODES"):
    MODES = [m for m in MODES if m[0] in os.environ["DIAG_MODES"].split(",")]


def run(path, D, bits, minibatch, epochs):
    oracle.lib().orc_set_diag_round(bits)
    c = CFG
    o = oracle.W2V(path, D, window=c["window"], negative=c["negative"], minibatch=minibatch, sample=c["sample"],
                   alpha=c["alpha"], lr=c["lr"], table_size=c["table"], storage_f32=True)
    o.init_rand(1, 2)
    o.train(epochs)
    oracle.lib().orc_set_diag_round(0)
    return o.get_params()


def main():
    tmp = "/tmp/diag_bfp"
    os.makedirs(tmp, exist_ok=True)
    cases = [("1 batch", corpus(os.path.join(tmp, "c40.txt"), lines=40, seed=83), 40, 1),
             ("2 batches", corpus(os.path.join(tmp, "c41.txt"), lines=41, seed=83), 40, 1),
             ("2 epochs", corpus(os.path.join(tmp, "c2.txt")), CFG["minibatch"], 2)]
    for name, path, mb, ep in cases:
        for D in (300, 100):
            ref = run(path, D, 0, mb, ep)
            for mname, bits in MODES:
                rel = rel_err(run(path, D, bits, mb, ep), ref)
                print("%-9s D=%d %-18s max %.3g  p99.99 %.3g" % (name, D, mname, rel.max(), np.quantile(rel, 0.9999)),
                      flush=True)


if __name__ == "__main__":
    main()
