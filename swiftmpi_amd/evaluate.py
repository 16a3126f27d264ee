"""Model-quality measures for trained tables (numpy, host side; evaluation
only — nothing here is on the training path).

cbow_objective: the CBOW negative-sampling log-likelihood the reference's
learn_instance ascends (apps/word2vec/word2vec_global.h:663-718): for a
sample of positions, neu1 = sum of the full-window context v rows, then
log sigmoid(neu1 . h_word) + sum over k seeded unigram^0.75 negatives of
log sigmoid(-neu1 . h_neg).  Higher is better; used to compare training
modes (lockstep vs pipelined, fast vs parity) on the same corpus."""
import numpy as np


def _log_sigmoid(x):
    return -np.logaddexp(0.0, -x)


def cbow_objective(rows, dim, vid_lines, counts, window=5, negatives=5, positions=4000, seed=0):
    """rows: [V, >=2*dim] array whose first 2*dim columns are [h | v] in vid
    order; vid_lines: list of int arrays (each line's tokens as vids);
    counts: word counts in vid order — negatives are drawn from count^0.75,
    the training distribution (word2vec_global.h:467-497)."""
    rows = np.asarray(rows, dtype=np.float64)
    V, D = rows.shape[0], dim
    h, v = rows[:, :D], rows[:, D:2 * D]
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(np.asarray(counts, dtype=np.float64) ** 0.75)
    cdf /= cdf[-1]
    lens = np.array([len(l) for l in vid_lines])
    cand = np.nonzero(lens >= 2)[0]
    total, n = 0.0, 0
    for _ in range(positions):
        li = int(cand[rng.integers(len(cand))])
        line = vid_lines[li]
        p = int(rng.integers(len(line)))
        ctx = [line[c] for c in range(max(0, p - window), min(len(line), p + window + 1)) if c != p]
        neu1 = v[ctx].sum(0)
        total += _log_sigmoid(neu1 @ h[line[p]])
        neg = np.minimum(np.searchsorted(cdf, rng.random(negatives), side="right"), V - 1)
        total += _log_sigmoid(-(h[neg] @ neu1)).sum()
        n += 1
    return total / max(n, 1)


def text_vid_lines(path, vocab_keys, bkdr):
    """Lines of a text corpus as vid arrays (words split on ' ', keys by
    `bkdr`, vid = index of the key in vocab_keys); unknown words dropped."""
    index = {int(k): i for i, k in enumerate(vocab_keys)}
    out = []
    with open(path) as f:
        for line in f:
            vids = [index.get(bkdr(w)) for w in line.rstrip("\n").split(" ") if w]
            out.append(np.array([x for x in vids if x is not None], dtype=np.int64))
    return out
