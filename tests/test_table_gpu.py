"""The HBM parameter shard: pull / push / assign / export / dump / load."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pull_inserts_and_push_adagrad(lib, gpu):
    D = 8
    t = lib.Table("w2v", dim=D, capacity=1000, dtype="f64", learning_rate=0.7, init="hash", seed=3)
    keys = torch.tensor(np.random.default_rng(0).choice(2 ** 62, 300, replace=False), dtype=torch.int64,
                        device=gpu)
    v1 = t.pull(keys)
    assert t.size() == 300 and v1.shape == (300, 2 * D)
    assert (v1.abs() <= 0.5 / D).all() and v1.abs().sum() > 0
    v2 = t.pull(keys)  # hits return the same rows
    assert torch.equal(v1, v2)
    g = torch.randn(300, 2 * D, dtype=torch.float64, device=gpu) * 1e-2
    rows0 = t.export(keys)
    t.push(keys, g)
    rows1 = t.export(keys)
    h, v = rows0[:, :D], rows0[:, D:2 * D]
    gh, gv = g[:, :D], g[:, D:]
    h2 = gh * gh
    lr = float(np.float32(0.7))  # float initial_learning_rate promoted to double
    exp_h = h + (gh * lr) / torch.sqrt(h2 + float(np.float32(1e-6)))
    assert torch.allclose(rows1[:, :D], exp_h, rtol=1e-12, atol=0)
    assert torch.allclose(rows1[:, 2 * D:3 * D], h2, rtol=1e-12, atol=0)


def test_push_unknown_key_is_error(lib, gpu):
    t = lib.Table("lr", capacity=10, dtype="f32")
    k = torch.tensor([5, 6], dtype=torch.int64, device=gpu)
    t.pull(k[:1])
    with pytest.raises(lib.SwpsError) as e:
        t.push(k, torch.zeros(2, 1, dtype=torch.float32, device=gpu))
    assert "BADKEY" in str(e.value)


def test_capacity_exhausted_is_error(lib, gpu):
    t = lib.Table("lr", capacity=4, dtype="f32")
    with pytest.raises(lib.SwpsError) as e:
        t.pull(torch.arange(10, dtype=torch.int64, device=gpu))
    assert "OOM" in str(e.value)


def test_full_table_overflow_key_is_never_a_row(lib, gpu):
    """A key whose insert found the table full owns a hash slot but no row
    (kFullRow): a later pull or push of it must fail as a miss, never read
    or write row 0xFFFFFFFE, and the stored keys keep working."""
    t = lib.Table("lr", capacity=4, dtype="f32")
    with pytest.raises(lib.SwpsError):
        t.pull(torch.arange(10, dtype=torch.int64, device=gpu))
    stored = sorted(int(x) for x in t.keys())
    assert len(stored) == 4
    over = [x for x in range(10) if x not in stored]
    ko = torch.tensor(over[:1], dtype=torch.int64, device=gpu)
    with pytest.raises(lib.SwpsError) as e:
        t.push(ko, torch.ones(1, 1, dtype=torch.float32, device=gpu))
    assert "BADKEY" in str(e.value)
    with pytest.raises(lib.SwpsError):
        t.pull(ko)
    ks = torch.tensor(stored, dtype=torch.int64, device=gpu)
    before = t.pull(ks).clone()
    t.push(ks, torch.full((4, 1), 0.5, dtype=torch.float32, device=gpu))
    after = t.pull(ks)
    assert torch.isfinite(after).all() and not torch.equal(before, after)


def test_w2v_dump_format_and_sharded_load(lib, gpu, tmp_path):
    D = 4
    t = lib.Table("w2v", dim=D, capacity=100, dtype="f32", init="hash", seed=1)
    keys = torch.arange(1, 51, dtype=torch.int64, device=gpu)
    t.pull(keys)
    path = str(tmp_path / "out.txt")
    t.dump(path)
    lines = open(path).read().strip().split("\n")
    assert len(lines) == 50
    key, v, h = lines[0].split("\t")
    assert len(v.split(" ")) == D and len(h.split(" ")) == D
    # server.h:49-62: each server keeps only the keys its hash-frag node owns
    fm = lib.hashfrag_table(1000, 2)
    owners = lib.to_node_id(np.arange(1, 51, dtype=np.uint64), 1000, fm)
    for node in (1, 2):
        t2 = lib.Table("w2v", dim=D, capacity=100, dtype="f32")
        t2.load(path, frag_num=1000, world=2, node_id=node)
        assert sorted(int(k) for k in t2.keys()) == [i + 1 for i in range(50) if owners[i] == node]


def test_duplicate_keys_in_one_pull_share_a_row(lib, gpu):
    """The reference's key sets are std::unordered_set (distinct); a caller
    that repeats a key in one pull still gets one row for it — the inserting
    thread publishes the row after its CAS, and a duplicate waits for it —
    never a spurious zero row or an OOM."""
    t = lib.Table("w2v", dim=8, capacity=64, dtype="f32", init="hash", seed=7)
    base = torch.arange(100, 132, dtype=torch.int64, device=gpu)
    keys = torch.cat([base, base, base[:7]])  # each key 2-3 times, in one call
    v = t.pull(keys)
    assert t.size() == 32
    assert torch.equal(v[:32], v[32:64]) and torch.equal(v[:7], v[64:])
    assert v.abs().sum(dim=1).min() > 0  # every copy got the initialised row
    assert torch.equal(t.pull(base), v[:32])


def test_flcg_init_continues_gen_float_in_call_order(lib, gpu):
    """SWPS_INIT_FLCG (LRPullAccessMethod::init_param = global_random().gen_float(),
    lr.cpp:48-50): the new keys of each pull take the next draws of the float
    LCG in the order the call lists them; keys already held keep their value
    and draw nothing; the stream continues across calls (and blocks of keys)."""
    import torch
    from test_lr_gpu import _gen_float_draws
    t = lib.Table("lr", capacity=1 << 16, dtype="f32", learning_rate=0.05, init="flcg")
    rng = np.random.default_rng(4)
    k1 = rng.choice(1 << 40, 3000, replace=False).astype(np.int64) + 1
    k2 = np.concatenate([k1[::7], rng.choice(1 << 40, 1500, replace=False).astype(np.int64) + (1 << 41)])
    k2 = k2[rng.permutation(len(k2))]
    v1 = t.pull(torch.as_tensor(k1, device="cuda")).cpu().numpy()[:, 0]
    v2 = t.pull(torch.as_tensor(k2, device="cuda")).cpu().numpy()[:, 0]
    draws = _gen_float_draws(3000 + 1500)
    assert np.array_equal(v1, draws[:3000])
    old = {int(k): x for k, x in zip(k1, v1)}
    new = [i for i, k in enumerate(k2) if int(k) not in old]
    assert len(new) == 1500
    assert np.array_equal(v2[new], draws[3000:])
    assert all(v2[i] == old[int(k)] for i, k in enumerate(k2) if int(k) in old)
    with pytest.raises(lib.SwpsError):
        lib.Table("w2v", dim=8, capacity=64, init="flcg")  # LR layout only
