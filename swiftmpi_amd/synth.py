"""Synthetic workloads of SURVEY.md §8(d) (there is no network for text8 or
Criteo): the bench and the tests generate their inputs here.  Data
generation only — nothing in this module is on the compute path."""
import numpy as np


def zipf_tokens(tokens, vocab, line_len, seed, s=1.0, progress=False):
    """Zipf(s) over `vocab` word ids, `tokens` tokens in lines of `line_len`
    (config 1/2/4: the text8 stand-in).  Returns (ids uint32, line_off uint64).
    progress: a line on stderr per 16M tokens (long generations stay visibly alive)."""
    import sys
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(1.0 / np.arange(1, vocab + 1) ** s)
    cdf /= cdf[-1]
    ids = np.empty(tokens, dtype=np.uint32)
    step = 1 << 24
    for a in range(0, tokens, step):
        b = min(tokens, a + step)
        ids[a:b] = np.minimum(np.searchsorted(cdf, rng.random(b - a), side="right"), vocab - 1)
        if progress:
            print("synth: %d / %d tokens" % (b, tokens), file=sys.stderr, flush=True)
    off = np.arange(0, tokens, line_len, dtype=np.uint64)
    off = np.append(off, np.uint64(tokens))
    return ids, off


CRITEO_SLOTS = 39
CRITEO_NUMERIC = 13
CRITEO_BITS = 24


def criteo(rows, seed=3, bits=CRITEO_BITS):
    """Criteo-shaped hashed sparse features (config 3): 39 features per row,
    13 numeric slots with values in (0, 1], 26 categorical slots with value 1;
    slot s's category ~ Zipf(1.2) capped at card_s in [10, 1e6]; feature =
    (cat*2654435761 + s*40503) mod 2^bits; label ~ Bernoulli(sigmoid(0.3 *
    sum w_true[f] x_f)) with w_true ~ N(0, 0.5^2).
    Returns (labels f32, row_off u64, feat u32, vals f32)."""
    rng = np.random.default_rng(seed)
    card = np.round(10 ** rng.uniform(1, 6, CRITEO_SLOTS)).astype(np.int64)
    mask = (1 << bits) - 1
    feat = np.empty((rows, CRITEO_SLOTS), dtype=np.uint32)
    vals = np.ones((rows, CRITEO_SLOTS), dtype=np.float32)
    for s in range(CRITEO_SLOTS):
        cdf = np.cumsum(1.0 / np.arange(1, card[s] + 1) ** 1.2)
        cdf /= cdf[-1]
        cat = np.searchsorted(cdf, rng.random(rows), side="right").astype(np.uint64)
        feat[:, s] = ((cat * np.uint64(2654435761) + np.uint64(s * 40503)) & np.uint64(mask)).astype(np.uint32)
        if s < CRITEO_NUMERIC:
            vals[:, s] = (1.0 - rng.random(rows)).astype(np.float32)
    w_true = rng.normal(0.0, 0.5, 1 << bits).astype(np.float32)
    z = 0.3 * (w_true[feat] * vals).sum(1)
    labels = (rng.random(rows) < 1.0 / (1.0 + np.exp(-z))).astype(np.float32)
    row_off = np.arange(0, rows * CRITEO_SLOTS + 1, CRITEO_SLOTS, dtype=np.uint64)
    return labels, row_off, feat.ravel(), vals.ravel()


def analogy_corpus(path, entities=40, relations=4, lines=3000, segments=12, ctx_words=3, noise_vocab=400,
                   seed=11):
    """A planted-analogy corpus (text8 and questions-words.txt are not
    available offline): target words "e<i>_r<j>" occur amid entity-context
    words "ce<i>_<k>", relation-context words "cr<j>_<k>" and Zipfian noise,
    so a trained v vector of e<i>_r<j> is close to an entity part plus a
    relation part and  v(e_a r_y) - v(e_a r_x) + v(e_b r_x) ~ v(e_b r_y).
    Writes `lines` lines of `segments` segments each; returns the question
    list [(a, b, c, expected)] of word strings."""
    rng = np.random.default_rng(seed)
    zp = 1.0 / np.arange(1, noise_vocab + 1)
    zp /= zp.sum()
    with open(path, "w") as f:
        for _ in range(lines):
            words = []
            for _ in range(segments):
                i, j = int(rng.integers(entities)), int(rng.integers(relations))
                seg = ["ce%d_%d" % (i, k) for k in rng.integers(0, ctx_words, 2)]
                seg += ["cr%d_%d" % (j, k) for k in rng.integers(0, ctx_words, 2)]
                seg += ["n%d" % k for k in rng.choice(noise_vocab, 2, p=zp)]
                rng.shuffle(seg)
                seg.insert(3, "e%d_r%d" % (i, j))
                words += seg
            f.write(" ".join(words) + "\n")
    qs = []
    for a in range(entities):
        for b in range(entities):
            if a == b:
                continue
            for x in range(relations):
                for y in range(relations):
                    if x != y:
                        qs.append(("e%d_r%d" % (a, x), "e%d_r%d" % (a, y), "e%d_r%d" % (b, x), "e%d_r%d" % (b, y)))
    return qs


def analogy_accuracy(vecs, index, questions, candidates):
    """questions-words style top-1 accuracy: for (a, b, c, d) predict
    argmax cos(x, b - a + c) over `candidates` (word strings) excluding a, b,
    c.  vecs: [V, D] word vectors; index: word -> row."""
    cand = np.array([index[w] for w in candidates])
    m = vecs[cand].astype(np.float64)
    m /= np.linalg.norm(m, axis=1, keepdims=True) + 1e-30
    pos = {int(r): k for k, r in enumerate(cand)}
    ok = 0
    for a, b, c, d in questions:
        q = vecs[index[b]] - vecs[index[a]] + vecs[index[c]]
        s = m @ q
        for w in (a, b, c):
            s[pos[index[w]]] = -np.inf
        ok += int(cand[int(np.argmax(s))] == index[d])
    return ok / max(len(questions), 1)
