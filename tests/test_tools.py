"""Host-side measurement tooling (no GPU): scripts/pmc_summary.py's HBM-byte
arithmetic on synthetic rocprofv3 counter CSVs, and bench.py's lookup of the
committed summary for a workload."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _csv(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w") as f:
        f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
        for r in rows:
            f.write("%d,\"%s\",%s,%s\n" % r)


def test_pmc_summary_read_requests_by_size(tmp_path):
    k = "void (anonymous namespace)::k_push_b<1, 1, 0, 8, false, 4>((anonymous namespace)::PushArgs<float, float>)"
    rd, wr, fe = str(tmp_path / "rd"), str(tmp_path / "wr"), str(tmp_path / "fe")
    rows = []
    for i in range(3):  # 3 launches; the last 2 are the window
        rows += [(i, k, "TCC_EA0_RDREQ_32B_sum", 10 * (i + 1)), (i, k, "TCC_EA0_RDREQ_64B_sum", 20 * (i + 1)),
                 (i, k, "TCC_EA0_RDREQ_128B_sum", 1000 * (i + 1)), (i, k, "TCC_EA0_RDREQ_sum", 1030 * (i + 1))]
    _csv(rd, rows)
    _csv(wr, [(i, k, "WRITE_SIZE", 4.0 * (i + 1)) for i in range(3)])
    _csv(fe, [(i, k, "FETCH_SIZE", 64.0 * (i + 1)) for i in range(3)])
    out = str(tmp_path / "s.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), out, rd, wr, fe, "--last", "2",
                        "--config", '{"app": "w2v"}'], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    s = json.load(open(out))
    e = s["kernels"]["k_push_b<1, 1, 0, 8, false, 4>"]
    # launches 2 and 3 averaged: 32*25 + 64*50 + 128*2500 read, 4*2.5 KiB written
    assert e["read_bytes"] == 32 * 25 + 64 * 50 + 128 * 2500
    assert e["write_bytes"] == 10.0 * 1024
    assert e["hbm_bytes"] == e["read_bytes"] + e["write_bytes"]
    assert abs(e["fetch_ratio"] - e["read_bytes"] / (160.0 * 1024)) < 1e-12
    assert s["config"] == {"app": "w2v"}


def test_pmc_summary_sq_wave_state_fractions(tmp_path):
    """An SQ pass (scripts/gpu_sq.sh): WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as fractions
    of WAVE_CYCLES (they partition it), cycles and instructions per wave; no byte fields."""
    k = "void (anonymous namespace)::k_lr_tiles<6, 256>((anonymous namespace)::LrReduce, (anonymous namespace)::LrTiles)"
    sq = str(tmp_path / "sq")
    rows = []
    for i in range(2):
        rows += [(i, k, "SQ_WAVES", 100), (i, k, "SQ_WAVE_CYCLES", 10000), (i, k, "SQ_WAIT_ANY", 5000),
                 (i, k, "SQ_WAIT_INST_ANY", 3000), (i, k, "SQ_ACTIVE_INST_ANY", 2000), (i, k, "SQ_INSTS_VALU", 600),
                 (i, k, "SQ_INSTS_VMEM_RD", 30), (i, k, "SQ_BUSY_CYCLES", 9000)]
    _csv(sq, rows)
    out = str(tmp_path / "sq.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), out, sq, "--last", "2"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    e = json.load(open(out))["kernels"]["k_lr_tiles<6, 256>"]
    assert (e["parked_frac"], e["issue_stall_frac"], e["active_frac"]) == (0.5, 0.3, 0.2)
    assert e["quad_cycles_per_wave"] == 100.0 and e["valu_per_wave"] == 6.0 and e["vmem_rd_per_wave"] == 0.3
    assert e["hbm_bytes"] is None
    assert "parked 0.50" in r.stdout


def test_bench_pmc_lookup_matches_config_and_kernel_base_names(tmp_path, monkeypatch):
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r03_pmc_x.json").write_text(json.dumps({
        "config": {"app": "w2v", "mode": "bfp32", "sharded": False},
        "kernels": {"k_gather_b<1, 1, 0, 8>": {"hbm_bytes": 5.0}, "k_push_b<1, 1, 0, 8, false, 4>": {"hbm_bytes": 7.0},
                    "k_forward_b<1, 1, 0, 4>": {"hbm_bytes": 11.0}, "k_gather_t<1, 8>": {"hbm_bytes": 100.0}}}))
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    res, src = b.pmc_traffic({"app": "w2v", "mode": "bfp32", "sharded": False},
                             {"sum": ("k_gather_b", "k_combine_b", "k_push_b"), "forward": ("k_forward_b",)})
    assert res == {"sum": 12.0, "forward": 11.0} and "r03_pmc_x.json" in src
    res, src = b.pmc_traffic({"app": "w2v", "mode": "bfp32", "sharded": True}, {"sum": ("k_gather_b",)})
    assert res == {"sum": None} and src is None  # a sharded line never borrows the unsharded counters


def test_bench_lr_tile_pieces_matches_a_loop_restatement():
    """bench.lr_tile_pieces (the LR row-tile path's pieces and partials, for its algorithmic
    bytes) against a plain loop over the same definition: records in (tile, key) order, row
    order inside a key; blocks of `chunk` records per tile; a piece = a key's records in one
    block; partials = the pieces of keys with more than one."""
    import importlib.util
    import numpy as np
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 9, 700)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    f = (rng.zipf(1.3, int(off[-1])) % 50).astype(np.uint32)
    for r0, r1, tb, ch in ((0, 700, 6, 16), (100, 613, 5, 7), (0, 700, 12, 1024)):
        recs = []
        for r in range(r0, r1):
            for c in range(int(off[r]), int(off[r + 1])):
                recs.append((((r - r0) >> tb), int(f[c]), r))
        recs.sort(key=lambda t: (t[0], t[1], t[2]))
        pieces, seen, start, prev = [], {}, {}, None
        for pos, (t, k, _) in enumerate(recs):
            start.setdefault(t, pos)
            blk = (pos - start[t]) // ch
            if (t, blk, k) != prev:
                pieces.append(k)
                prev = (t, blk, k)
        for k in pieces:
            seen[k] = seen.get(k, 0) + 1
        exp = (len(pieces), sum(n for n in seen.values() if n > 1))
        assert b.lr_tile_pieces(f, off, r0, r1, tile_bits=tb, chunk=ch) == exp


def test_bench_refuses_world_size_that_differs_from_gpus():
    """The driver's contract: `--gpus N` is the world.  A launcher whose
    WORLD_SIZE disagrees is refused (rc 2) before anything touches the GPU."""
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 2 and "--gpus 1" in r.stderr


def test_bench_launcher_spawns_ranks(tmp_path, monkeypatch):
    """Without WORLD_SIZE, `--gpus N` starts N rank processes of bench.py with
    torch.distributed.run's variables (a stand-in script records them) and
    returns the first failing rank's code."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    stub = tmp_path / "stub.py"
    stub.write_text("import json, os, sys\n"
                    "d = {k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}\n"
                    "open(os.path.join(%r, 'r%%s.json' %% d['RANK']), 'w').write(json.dumps([d, sys.argv[1:]]))\n"
                    "sys.exit(3 if d['RANK'] == '2' else 0)\n" % str(tmp_path))
    monkeypatch.setattr(b.os.path, "abspath", lambda p: str(stub) if p == b.__file__ else os.path.realpath(p))
    rc = b.launch_ranks(3, ["--gpus", "3", "--steps", "2"])
    assert rc == 3
    seen = [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(3)]
    assert [d["RANK"] for d, _ in seen] == ["0", "1", "2"] and {d["WORLD_SIZE"] for d, _ in seen} == {"3"}
    assert {d["MASTER_ADDR"] for d, _ in seen} == {"127.0.0.1"} and len({d["MASTER_PORT"] for d, _ in seen}) == 1
    assert all(a == ["--gpus", "3", "--steps", "2"] for _, a in seen)
