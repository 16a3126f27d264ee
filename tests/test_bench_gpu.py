"""bench.py as the driver runs it, on the one-GPU box: `--gpus 2` starts two
rank processes itself (no external launcher), they share cuda:0 over the
library's TCP transport (RCCL refuses two ranks on one device), and rank 0
prints one line with n_gpus 2, the world-2 exchange block and — at every N —
the config-4, LR (config 3) and sent2vec (config 5) legs, each with its own
exchange accounting.  A rank that dies mid-run ends the command with rc != 0
within the deadline instead of leaving its sibling waiting in a collective."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SMALL = ["--steps", "2", "--warmup", "1", "--tokens", "1000000", "--vocab", "50000", "--minibatch", "200",
         "--no-cpu-baseline", "--no-parity-leg", "--b100-steps", "0", "--config1-steps", "0"]
LEGS = ["--config4-tokens", "2000000", "--config4-steps", "2", "--lr-batch", "4096", "--app-steps", "3",
        "--s2v-docs", "256"]


def _env(**kw):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **kw)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


def test_bench_gpus2_spawns_two_ranks(lib, gpu):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL + ["--no-app-legs"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = _line(r)
    print({k: out[k] for k in ("value", "n_gpus", "ms_per_step", "transport")}, out["exchange"])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["transport"] == "tcp" and out["transport_ranks"] == 2
    x = out["exchange"]
    assert x is not None and x["world"] == 2 and x["bytes_remote_per_step"] > 0 and x["a2a_per_step"] >= 2
    assert "key-sharded PS over 2 GPU(s)" in out["config"]["parallelism"]


def test_bench_gpus2_every_leg(lib, gpu):
    """The N > 1 line carries config 4 (key-sharded, frag_num 8000), LR (key-sharded over the
    library's communicator, frag 2000) and sent2vec (doc-sharded, replicas only) beside the
    headline, each with n_gpus 2 and its own exchange block."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL + LEGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = _line(r)
    c4, lr, s2 = out["config4"], out["lr"], out["s2v"]
    print({k: (v["value"], v["ms_per_step"]) for k, v in (("config4", c4), ("lr", lr), ("s2v", s2))})
    for leg in (c4, lr, s2):
        assert leg["n_gpus"] == 2 and leg["value"] > 0
    assert "frag_num 8000" in c4["config"]["parallelism"] and c4["transport_ranks"] == 2
    assert c4["exchange"]["world"] == 2 and c4["exchange"]["bytes_remote_per_step"] > 0
    assert "frag_num 2000" in lr["config"]["parallelism"] and lr["transport_ranks"] == 2
    assert lr["exchange"]["world"] == 2 and lr["exchange"]["bytes_remote_per_step"] > 0
    assert lr["config"]["end_to_end"]["value"] > 0 and lr["config"]["setup_s"]["load"] > 0
    assert "replicas only" in s2["config"]["parallelism"] and s2["config"]["end_to_end"]["value"] > 0


def test_bench_rank_killed_fails_fast(lib, gpu):
    """Rank 1 kills itself (SIGKILL) entering the LR leg: the command exits non-zero well
    within the deadline, and says which rank died."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL + LEGS
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=_env(SWPS_BENCH_FAULT="1:lr", SWPS_BENCH_DEADLINE_S="200",
                                               SWPS_COMM_TIMEOUT_S="30"),
                       capture_output=True, text=True, timeout=300)
    dt = time.time() - t0
    print(dt, r.returncode, r.stderr[-1500:])
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr and "SWPS_BENCH_FAULT" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert dt < 260


def test_bench_gpus1_lr_sharded_base_forms(lib, gpu):
    """At N = 1 the LR leg carries its world-1 sharded base point in both forms: the full protocol
    (`lr.sharded_world1`, SWPS_PULL_IN_PLACE=0 — what every rank runs at N > 1) and the library
    driver's in-place default (`.in_place`); the s2v leg's value is the load-inclusive single pass,
    its re-train the `steady_state` sub-field."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + SMALL + LEGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = _line(r)
    lr, s2 = out["lr"], out["s2v"]
    q = lr["sharded_world1"]
    print(lr["ms_per_step"], q["ms_per_step"], q["in_place"]["ms_per_step"], s2["value"])
    assert q["value"] > 0 and q["in_place"]["value"] > 0 and "SWPS_PULL_IN_PLACE=0" in q["note"]
    assert "key-sharded PS over 1 GPU(s)" in q["parallelism"]
    assert s2["value"] == s2["config"]["end_to_end"]["value"] and s2["config"]["steady_state"]["value"] > 0
